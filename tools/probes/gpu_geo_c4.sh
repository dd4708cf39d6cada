# C4 on both segmented geometries (run via gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/geo
for g in hex tri hex; do
  if [ $g = tri ]; then export HPGQ_TRI_GEO=tri; else unset HPGQ_TRI_GEO; fi
  timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/geo/c4_$g.json 2> gpurun_out/geo/c4_$g.err || exit 4
done
