"""Helpers to drive the C host CLI (hpg-fastq_amd/hpg-fastq) from tests."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "hpg-fastq_amd", "hpg-fastq")


def run_cli(args, check=True, timeout=300, env=None):
    r = subprocess.run([CLI] + [str(a) for a in args], capture_output=True, text=True,
                       timeout=timeout, env=None if env is None else dict(os.environ, **env))
    if check and r.returncode != 0:
        raise AssertionError(f"hpg-fastq {args} -> {r.returncode}\n{r.stdout}\n{r.stderr}")
    return r


def print_params(cmd, *flags):
    r = run_cli([cmd, "--print-params"] + list(flags))
    d = {}
    for tok in r.stdout.split():
        k, v = tok.split("=")
        d[k] = int(v)
    return d
