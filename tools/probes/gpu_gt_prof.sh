# round 3 GT probe: HBM bytes + instruction counts of the C4 edit kernel (prof_engine edit mode)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gtp
export TMPDIR=/tmp
A="python tools/prof_engine.py --mode ${MODE:-edit} --reads 12500000 --L 150 --iters 3"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/gtp/fetch -o run --output-format csv -- $A > gpurun_out/gtp/fetch.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH -d gpurun_out/gtp/sq1 -o run --output-format csv -- $A > gpurun_out/gtp/sq1.log 2>&1 || exit 3
python - <<'PY'
import csv, glob
for tag in ("fetch", "sq1"):
    f = glob.glob(f"gpurun_out/gtp/{tag}/**/run_counter_collection.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    agg = {}
    for r in rows:
        if "engine_tri" not in r["Kernel_Name"]:
            continue
        agg.setdefault((r["Dispatch_Id"], r["Counter_Name"]), 0.0)
        agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    last = max(int(d) for d, _ in agg) if agg else None
    print(tag, {c: v for (d, c), v in agg.items() if int(d) == last})
PY
