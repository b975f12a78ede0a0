#!/usr/bin/env python3
"""Microbenchmark of the scheduling scan alone (k10s_schedule_one_batch): R independent
schedule_one calls over N-node caches resident in HBM.  Algorithmic bytes per call = 12*N + 12
(u32 cpu + u64 ram per node + the pod request); reports GB/s against the 8 TB/s HBM peak."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problems", type=int, default=8192)
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch
    from kubernetriks_amd.native import lib
    L = lib()
    R, N = a.problems, a.nodes
    stride = (N + 63) // 64 * 64
    g = torch.Generator().manual_seed(0)
    dev = torch.device("cuda:0")
    cpu = torch.randint(1000, 64000, (R * stride,), generator=g, dtype=torch.int32).to(dev)
    ram = torch.randint(1 << 30, 1 << 37, (R * stride,), generator=g, dtype=torch.int64).to(dev)
    bits = torch.full((R * stride // 64,), -1, dtype=torch.int64, device=dev)
    rc = torch.full((R,), 500, dtype=torch.int32, device=dev)
    rr = torch.full((R,), 1 << 29, dtype=torch.int64, device=dev)
    on = torch.empty(R, dtype=torch.int32, device=dev)
    st = torch.empty(R, dtype=torch.int32, device=dev)

    def launch():
        rcode = L.k10s_schedule_one_batch(cpu.data_ptr(), ram.data_ptr(), bits.data_ptr(), N, stride, rc.data_ptr(),
                                          rr.data_ptr(), 1.0, R, on.data_ptr(), st.data_ptr(), None)
        assert rcode == 0
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        launch()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    bytes_per = R * (12.0 * N + 12.0)
    out = {"kernel": "k10s_schedule_kernel", "problems": R, "nodes": N, "ms_per_launch": ms,
           "achieved_GBps": bytes_per / (ms * 1e-3) / 1e9, "frac_of_8TBps": bytes_per / (ms * 1e-3) / 8e12,
           "nodes_per_s": R * N / (ms * 1e-3), "attempts_per_s": R / (ms * 1e-3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
