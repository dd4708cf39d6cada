"""A/B of the stored-output writer settings on one GPU box: one synthetic
FASTQ (tools/fqgen.c, bench.py's e2e file: 20M x 150 bp in /dev/shm, generated
on the GPU's NUMA CPUs), then `hpg-fastq filter` / `edit` with each variant's
extra flags, the variants alternating over REPS rounds so clock and page-cache
drift spreads evenly.  Prints one JSON line per variant/command with the CLI's
own Mreads/s per run (median, min) and the writer the trace line names.

  python tools/writer_ab.py OUT.json [--reps 3] [--reads N] \
      'name=--flag v --flag2 v2' 'name2=' ...
"""
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (numa_cpus / omp_threads / E2E_READS)


def main():
    a = sys.argv[1:]
    out_json = a.pop(0)
    reps, reads = 3, bench.E2E_READS
    while a and a[0].startswith("--"):
        k, v = a.pop(0), a.pop(0)
        if k == "--reps":
            reps = int(v)
        elif k == "--reads":
            reads = int(v)
    variants = [(s.split("=", 1)[0], s.split("=", 1)[1].split()) for s in a]
    cli = os.path.join(ROOT, "hpg-fastq_amd", "hpg-fastq")
    tmp = tempfile.mkdtemp(prefix="hpgq_wab_")
    gen = os.path.join(tmp, "fqgen")
    fq = f"/dev/shm/hpgq_wab_{os.getpid()}.fq"
    outd = f"/dev/shm/hpgq_wab_out_{os.getpid()}"
    bench._load_hpgfastq()
    cpus = bench.numa_cpus(0)
    share = sorted(cpus)[:bench.omp_threads(len(cpus) or 16)] if cpus else None
    nthr = str(len(share) if share else 16)
    flags = {"filter": ["--read-quality-range", "20,", "--read-length-range", "50,"],
             "edit": ["--left-length", "10", "--left-quality-range", "20,", "--right-length", "30",
                      "--right-quality-range", "20,"]}
    res = {}
    try:
        subprocess.run(["gcc", "-O2", "-fopenmp", os.path.join(ROOT, "tools", "fqgen.c"), "-o", gen],
                       check=True, timeout=120)
        subprocess.run([gen, fq, str(reads), "150", "2", ",".join(map(str, share or []))], check=True,
                       timeout=300, env=dict(os.environ, OMP_NUM_THREADS=nthr))
        for rep in range(reps + 1):          # round 0: warm-up, not counted
            for name, extra in variants:
                for cmd, fl in flags.items():
                    shutil.rmtree(outd, ignore_errors=True)
                    os.makedirs(outd)
                    r = subprocess.run([cli, cmd, "-f", fq, "-o", outd, *fl, "--gpus", "1", "--gpu", "0",
                                        "--num-threads", nthr, *extra],
                                       capture_output=True, text=True, timeout=300)
                    m = re.search(r"= ([0-9.]+) Mreads/s", r.stdout)
                    w = re.search(r"Output writer\s*:\s*(.+)", r.stdout)
                    rec = res.setdefault(f"{name} {cmd}", {"flags": extra, "runs": [], "rc": []})
                    rec["writer"] = w.group(1).strip() if w else None
                    if r.returncode or not m:
                        rec["rc"].append(r.returncode)
                        rec["err"] = (r.stderr or r.stdout)[-300:]
                        continue
                    if rep:
                        rec["runs"].append(float(m.group(1)))
                    print(name, cmd, rep, m.group(1), flush=True)
    finally:
        for f in (fq,):
            try:
                os.remove(f)
            except OSError:
                pass
        shutil.rmtree(outd, ignore_errors=True)
        shutil.rmtree(tmp, ignore_errors=True)
    for k, v in res.items():
        if v["runs"]:
            s = sorted(v["runs"])
            v["median"], v["min"] = s[len(s) // 2], s[0]
        print(k, json.dumps(v), flush=True)
    json.dump(res, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main()
