"""Host round trip of one tiny kernel + torch.cuda.synchronize(), with the HIP device flags
given on the command line (0 auto, 1 spin, 2 yield, 4 blocking sync) set before torch touches
the device: how much of the driver's 20-step window is launch and wake-up latency."""
import ctypes, sys, time
import numpy as np

flags = int(sys.argv[1]) if len(sys.argv) > 1 else -1
if flags >= 0:
    hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags", flags, "->", hip.hipSetDeviceFlags(ctypes.c_uint(flags)))
import torch
x = torch.zeros(1, device="cuda")
for _ in range(50):
    x.add_(1)
torch.cuda.synchronize()
for name, n in (("1 kernel", 1), ("8 kernels", 8)):
    ts = []
    for _ in range(300):
        t0 = time.perf_counter()
        for _ in range(n):
            x.add_(1)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts = np.array(ts) * 1e6
    print(f"flags {flags} {name}: median {np.median(ts):.1f} us  p10 {np.percentile(ts, 10):.1f}  p90 {np.percentile(ts, 90):.1f}")
