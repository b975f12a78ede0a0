"""The scheduling scan alone (k10s_schedule_one_batch): R independent schedule_one calls over
N-node caches resident in HBM, timed with HIP events on the launch stream.  Algorithmic bytes per
call = 12*N + 12 (u32 cpu + u64 ram per node + the pod request); reported against
the 8 TB/s HBM peak.  Used by bench.py (the "scheduling_kernel" object) and tools/bench_scan.py."""
from __future__ import annotations

HBM_PEAK = 8.0e12


def measure(problems: int = 8192, nodes: int = 4096, iters: int = 20, device: int = 0) -> dict:
    import torch
    from .native import lib
    L = lib()
    R, N = problems, nodes
    stride = (N + 63) // 64 * 64
    g = torch.Generator().manual_seed(0)
    dev = torch.device("cuda", device)
    # every node present and fitting (the C3 steady state): a full scan per call
    cpu = torch.randint(1000, 64000, (R * stride,), generator=g, dtype=torch.int32).to(dev)
    ram = torch.randint(1 << 30, 1 << 37, (R * stride,), generator=g, dtype=torch.int64).to(dev)
    bits = torch.full((R * stride // 64,), -1, dtype=torch.int64, device=dev)
    rc = torch.full((R,), 500, dtype=torch.int32, device=dev)
    rr = torch.full((R,), 1 << 29, dtype=torch.int64, device=dev)
    on = torch.empty(R, dtype=torch.int32, device=dev)
    st = torch.empty(R, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def launch():
        rcode = L.k10s_schedule_one_batch(cpu.data_ptr(), ram.data_ptr(), bits.data_ptr(), N, stride, rc.data_ptr(),
                                          rr.data_ptr(), 1.0, R, on.data_ptr(), st.data_ptr(), stream.cuda_stream)
        if rcode != 0:
            raise RuntimeError(f"k10s_schedule_one_batch failed: {rcode}")
    for _ in range(3):
        launch()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        launch()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    if int((st != 0).sum()) != 0:
        raise RuntimeError("scan microbenchmark: a call did not place its pod")
    ms = e0.elapsed_time(e1) / iters
    bytes_per = R * (12.0 * N + 12.0)
    gbps = bytes_per / (ms * 1e-3)
    del cpu, ram, bits
    return {"kernel": "k10s_schedule_kernel", "bound": "hbm", "problems": R, "nodes": N, "ms_per_launch": ms,
            "achieved": gbps / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": gbps / HBM_PEAK,
            "algorithmic_bytes_per_launch": bytes_per, "attempts_per_s": R / (ms * 1e-3)}
