# segmented-kernel A/B variants: recompile one geometry object with extra flags
# and link it with the other objects of the main build.
#   tools/probes/build_geo_ab.sh NAME GEO "-DFLAG=..." ...   (GEO 0 tri, 1 hex, 2 wide)
set -e
cd "$(dirname "$0")/../.."
name=$1; geo=$2; shift 2
out=hpg-fastq_amd/ab/build_$name
mkdir -p $out
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -ffp-contract=off \
  -I include -I hpg-fastq_amd/csrc -DHPGQ_GEO=$geo "$@" -c hpg-fastq_amd/csrc/hpgq_engine_geo.hip -o $out/geo.o
objs=$(ls hpg-fastq_amd/build/*.o | grep -v "hpgq_engine_geo$geo.o")
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -shared $objs $out/geo.o -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib -o hpg-fastq_amd/ab/libhpgq_$name.so
echo hpg-fastq_amd/ab/libhpgq_$name.so
