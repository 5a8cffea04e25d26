"""PMC summary (tools/pmc_summary.py output) -> profiles/pmc_traffic.json, the HBM bytes per
launch of the dominant kernel that bench.py reports as roofline.traffic.

Correction per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE
counts half the bytes of 16-B/lane streaming reads (global_load and buffer/global_load ...
lds alike) -> doubled; WRITE_SIZE is exact for 16-B/lane stores.  Both are in KiB.

    python tools/pmc_traffic.py gpurun_out/pmc/summary.json profiles/pmc_traffic.json
"""
import json
import os
import sys

KERNELS = {"f32": "bb::scan3_kernel<48", "bf16": "bb::scan2_kernel<unsigned short"}


def main(src, dst):
    summ = json.load(open(src))
    try:
        out = json.load(open(dst))
    except Exception:
        out = {}
    for dt, prefix in KERNELS.items():
        hit = [(k, v) for k, v in summ.items() if k.startswith(prefix)]
        if not hit:
            continue
        name, c = hit[0]
        fetch_kib, write_kib = c.get("FETCH_SIZE"), c.get("WRITE_SIZE")
        if fetch_kib is None or write_kib is None:
            continue
        out[dt] = {"gemm": {
            "kernel": name,
            "fetch_size_kib": fetch_kib, "write_size_kib": write_kib,
            "hbm_read_bytes_per_launch": 2.0 * fetch_kib * 1024,
            "hbm_write_bytes_per_launch": write_kib * 1024,
            "hbm_bytes_per_launch": 2.0 * fetch_kib * 1024 + write_kib * 1024,
            "correction": "FETCH_SIZE x2 (gfx950 16-B/lane reads), WRITE_SIZE x1; KiB -> bytes",
            "source": os.path.relpath(src, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))}}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
