"""Copy one GPU round's evidence from gpurun_out/<tag>/ into profiles/ (tracked):
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of `bench.py --no-cpu`
  profiles/<tag>_bench.json         the bench.py JSON line of the same round
  profiles/<tag>_pmc.json           per-dispatch PMC means (FETCH_SIZE / WRITE_SIZE ...) of libbrickrec kernels
  profiles/pmc_traffic.json         HBM bytes per launch of the dominant kernel (read by bench.py)

    python tools/collect_profiles.py r01
"""
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "prof", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
    for log in ("bench.log", "bench_bf16.log"):
        p = os.path.join(src, log)
        if os.path.exists(p):
            lines = [l for l in open(p) if l.startswith("{")]
            if lines:
                name = f"{tag}_bench.json" if log == "bench.log" else f"{tag}_bench_bf16.json"
                with open(os.path.join(dst, name), "w") as f:
                    f.write(lines[-1])
    summ = os.path.join(src, "pmc", "summary.json")
    if os.path.exists(summ):
        d = json.load(open(summ))
        mine = {k: v for k, v in d.items() if k.startswith("bb::")}
        with open(os.path.join(dst, f"{tag}_pmc.json"), "w") as f:
            json.dump(mine, f, indent=1)
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"),
                        os.path.join(dst, f"{tag}_pmc.json"), os.path.join(dst, "pmc_traffic.json")],
                       check=True, stdout=subprocess.DEVNULL)


if __name__ == "__main__":
    main(sys.argv[1])
