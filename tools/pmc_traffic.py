"""PMC summaries (tools/pmc_summary.py output, one per workload) -> profiles/pmc_traffic.json:
the HBM bytes per step of the scan launches that bench.py reports as roofline.traffic.

Correction per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE
counts half the bytes of 16-B/lane streaming reads (global_load and global_load ... lds
alike) -> doubled; WRITE_SIZE is exact for 16-B/lane stores.  Both are in KiB.

Per step = Σ over the scan kernels (mean bytes per dispatch × dispatches) ÷ dispatches of the
workload's once-per-step anchor kernel.

    python tools/pmc_traffic.py KEY summary.json [profiles/pmc_traffic.json]
    KEY: f32 (configs[1] scan3) | c3 (configs[2] hybrid) | c4 | c5 (sharded bf16)
"""
import json
import os
import sys

SCAN = ("bb::scan3_kernel", "bb::scan2_kernel", "bb::scan4_kernel", "bb::scan4_dual_kernel")
ANCHOR = {"f32": ("bb::select_list_kernel", "bb::select_kernel", "bb::scan3_kernel"), "c3": ("bb::finalize1_kernel",),
          "c4": ("bb::finalize_kernel", "bb::finalize1_kernel"), "c5": ("bb::finalize_kernel", "bb::finalize1_kernel")}


def main(key, src, dst):
    summ = json.load(open(src))
    try:
        out = json.load(open(dst))
    except Exception:
        out = {}
    anchor = None
    for a in ANCHOR[key]:
        hit = [v["_dispatches"] for k, v in summ.items() if k.startswith(a) and "_dispatches" in v]
        if hit:
            anchor = max(hit)
            break
    scans = {k: v for k, v in summ.items() if k.startswith(SCAN) and "FETCH_SIZE" in v and "WRITE_SIZE" in v}
    if not scans or not anchor:
        print("no scan kernels / anchor in", src)
        return
    rd = sum(2.0 * v["FETCH_SIZE"] * 1024 * v["_dispatches"] for v in scans.values()) / anchor
    wr = sum(v["WRITE_SIZE"] * 1024 * v["_dispatches"] for v in scans.values()) / anchor
    out[key] = {"gemm": {
        "kernels": {k: {"fetch_size_kib": v["FETCH_SIZE"], "write_size_kib": v["WRITE_SIZE"],
                        "dispatches": v["_dispatches"]} for k, v in scans.items()},
        "steps": anchor,
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr,
        "unit_note": "per step of the scan launches (one launch for configs[1])",
        "correction": "FETCH_SIZE x2 (gfx950 16-B/lane reads), WRITE_SIZE x1; KiB -> bytes",
        "source": os.path.relpath(src, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))}}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out[key], indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else
         os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json"))
