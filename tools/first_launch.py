"""Why the driver's 20-sweep line is slower per sweep: fresh record buffers vs reused ones.

    python tools/first_launch.py [C]
"""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from gibbs_student_t_amd.native import NativeSampler  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
K = 20
wl = bench.workload(2, 0, 1, C)
ns = NativeSampler(wl["ptas"], wl["cfgs"], 0)
ns.alloc(C)
ns.set_state(**wl["init"])
ns.sweep(5, seed=1)
s0 = 5
keys = ("x", "b", "z", "alpha", "pout", "theta", "nu")


def run(tag, rec):
    global s0
    ns.sweep(K, records=rec, seed=1, sweep0=s0)
    ns.synchronize()
    s0 += K
    print(f"{tag:44s} {ns.last_kernel_ms() / K * 1e3:7.1f} us/sweep", flush=True)


run("no records, after 5 sweeps", None)
run("fresh records (torch.empty)", ns.alloc_records(K, keys))
r = ns.alloc_records(K, keys)
for v in r.values():
    v.zero_()
torch.cuda.synchronize()
run("fresh records, zero-filled before", r)
run("same records again", r)
ns.sweep(3000, seed=1, sweep0=s0)
s0 += 3000
run("after 3000 burn-in, reused records", r)
run("after 3000 burn-in, fresh records", ns.alloc_records(K, keys))
r2 = ns.alloc_records(K, keys)
for v in r2.values():
    v.zero_()
torch.cuda.synchronize()
run("after 3000 burn-in, fresh zero-filled", r2)
