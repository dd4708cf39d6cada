# A/B baseline: libhpgq built from the kernel sources of a git revision
#   tools/probes/build_rev.sh REV NAME  -> hpg-fastq_amd/ab/NAME/libhpgq.so
# (not tracked; travels with gpurun; load with HPGQ_LIB_PATH=...)
set -e
cd "$(dirname "$0")/../.."
rev=$1; name=$2
tmp=$(mktemp -d)
mkdir -p $tmp/hpg-fastq_amd $tmp/include
git archive $rev hpg-fastq_amd/csrc include | tar -x -C $tmp
out=hpg-fastq_amd/ab/$name
mkdir -p $out
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -ffp-contract=off -I $tmp/include"
for f in $tmp/hpg-fastq_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  if [ "$b" = hpgq_engine_geo ]; then
    for g in 0 1 2; do /opt/rocm/bin/hipcc $F -DHPGQ_GEO=$g -c $f -o $out/${b}$g.o & done
  else
    /opt/rocm/bin/hipcc $F -c $f -o $out/$b.o &
  fi
done
for f in $tmp/hpg-fastq_amd/csrc/*.cpp; do g++ -O2 -std=c++17 -fPIC -ffp-contract=off -I $tmp/include -c $f -o $out/$(basename $f .cpp).o & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared $out/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o $out/libhpgq.so
rm -f $out/*.o
rm -rf $tmp
echo $out/libhpgq.so
