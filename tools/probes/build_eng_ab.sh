# engine-only A/B variants: recompile hpgq_engine.hip with extra flags, link with
# the other objects of the main build.  tools/build_eng_ab.sh NAME "-DFLAG=..." ...
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
out=hpg-fastq_amd/ab/build_$name
mkdir -p $out
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -Wno-inline-asm -ffp-contract=off \
  -I include -I hpg-fastq_amd/csrc "$@" -c hpg-fastq_amd/csrc/hpgq_engine.hip -o $out/hpgq_engine.o
objs=$(ls hpg-fastq_amd/build/*.o | grep -v hpgq_engine.o)
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -shared $objs $out/hpgq_engine.o -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib -o hpg-fastq_amd/ab/libhpgq_$name.so
echo hpg-fastq_amd/ab/libhpgq_$name.so
