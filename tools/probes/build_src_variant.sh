# A/B or timing-only variant of libhpgq from an edited copy of csrc:
#   build_src_variant.sh NAME [PATCH ...]      patches (against csrc/, -p1 from
#                                              a/ b/ file names) applied to the copy
#   build_src_variant.sh NAME < edit.py        no patch: a python snippet on stdin
#                                              rewrites the copy (cwd = the copy's csrc)
#   EXTRA_FLAGS="-DHPGQ_EDIT_ABL_NOTRIM=1" ... compile flags for the variant
#   -> hpg-fastq_amd/ab/NAME/libhpgq.so (not tracked; load with HPGQ_LIB_PATH)
# Timing-only switches (wrong results) live only in tools/probes/*.patch, never
# in the product source: c5_ablation.patch (HPGQ_C5_ABLATION 1-5, round 4),
# edit_notrim_ablation.patch (HPGQ_EDIT_ABL_NOTRIM 1-2).
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
tmp=$(mktemp -d)
mkdir -p $tmp/hpg-fastq_amd $tmp/include
cp -r hpg-fastq_amd/csrc $tmp/hpg-fastq_amd/ && cp include/hpgq.h $tmp/include/
if [ $# -gt 0 ]; then
  for p in "$@"; do patch -s -p1 -d $tmp/hpg-fastq_amd/csrc < "$p"; done
else
  (cd $tmp/hpg-fastq_amd/csrc && python3 -)
fi
out=hpg-fastq_amd/ab/$name
mkdir -p $out
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -ffp-contract=off -I $tmp/include $EXTRA_FLAGS"
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
