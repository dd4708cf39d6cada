# segmented-kernel A/B variants over all three geometries: recompile every
# geometry object with extra flags and link them with the other objects of the
# main build.   tools/probes/build_geoall_ab.sh NAME "-DFLAG=..." ...
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
out=hpg-fastq_amd/ab/build_$name
mkdir -p $out
for geo in 0 1 2; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -ffp-contract=off \
    -I include -I hpg-fastq_amd/csrc -DHPGQ_GEO=$geo "$@" -c hpg-fastq_amd/csrc/hpgq_engine_geo.hip -o $out/geo$geo.o &
done
wait
objs=$(ls hpg-fastq_amd/build/*.o | grep -v "hpgq_engine_geo[012].o")
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -shared $objs $out/geo0.o $out/geo1.o $out/geo2.o -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib -o hpg-fastq_amd/ab/libhpgq_$name.so
echo hpg-fastq_amd/ab/libhpgq_$name.so
