# A/B variant of libhpgq with extra compile flags (e.g. -DHPGQ_PE_WAVES=2):
#   tools/probes/build_variant.sh NAME FLAGS...  -> hpg-fastq_amd/ab/NAME/libhpgq.so
# (not tracked; travels with gpurun; load with HPGQ_LIB_PATH=...)
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
out=hpg-fastq_amd/ab/$name
mkdir -p $out
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -ffp-contract=off -I include"
for f in hpg-fastq_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  if [ "$b" = hpgq_engine_geo ]; then
    for g in 0 1 2; do /opt/rocm/bin/hipcc $F "$@" -DHPGQ_GEO=$g -c $f -o $out/${b}$g.o & done
  else
    /opt/rocm/bin/hipcc $F "$@" -c $f -o $out/$b.o &
  fi
done
for f in hpg-fastq_amd/csrc/*.cpp; do g++ -O2 -std=c++17 -fPIC -ffp-contract=off -I include -c $f -o $out/$(basename $f .cpp).o & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared $out/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o $out/libhpgq.so
rm -f $out/*.o
echo $out/libhpgq.so
