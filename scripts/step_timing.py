"""Round-5 timing of one call shape for the scripts (as bench.py): a 0.2-s
clock warm-up (profiles/r02c_clock_ramp.txt), then K back-to-back calls with
no per-launch events, bracketed by HIP events on the calling stream -- an
event pair around every launch idles the GPU ~10 us per launch
(profiles/r05h_event_gap_trace.json) -- and, in a second pass, the per-launch
event pairs (tcsc_hip_set_timing) for the kernel-only figure of rounds <= 4.
When a call is one launch (tcsc_hip_call_launches) the stream time per call
is that kernel's duration."""
import time


def time_calls(h, X, b, Y, steps, warm_s=0.2):
    import torch
    t_end = time.perf_counter() + warm_s
    while time.perf_counter() < t_end:
        for _ in range(4):
            h.gemm_torch(X, b, Y)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        h.gemm_torch(X, b, Y)
    e1.record()
    torch.cuda.synchronize()
    step_ms = e0.elapsed_time(e1) / steps
    h.set_timing(True)
    h.kernel_time(reset=True)
    for _ in range(steps):
        h.gemm_torch(X, b, Y)
    torch.cuda.synchronize()
    ms, n = h.kernel_time(reset=True)
    h.set_timing(False)
    return {"step_ms": step_ms, "event_pair_kernel_ms": ms / max(n, 1),
            "launches": h.call_launches(X, X.shape[0])}
