# build libhpgq variants for A/B timing: tools/build_ab.sh NAME "-DFLAG=..." ...
# -> hpg-fastq_amd/ab/libhpgq_NAME.so (not tracked; travels with gpurun)
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
out=hpg-fastq_amd/ab/build_$name
mkdir -p $out
for f in hpg-fastq_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -Wno-inline-asm -ffp-contract=off \
    -I include -I hpg-fastq_amd/csrc "$@" -c $f -o $out/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -shared $out/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o hpg-fastq_amd/ab/libhpgq_$name.so
echo hpg-fastq_amd/ab/libhpgq_$name.so
