"""Probe: does running the fill of one batch concurrently with the eval of another (two
streams, two resident traces) beat running them back to back? Prints wall ms per
fill+eval pair for both schedules at the fill grid given by B2F_FILL_WGS."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "zk-odst_amd"))


def main():
    import torch

    import b2f
    from b2f import synth

    n = int(os.environ.get("N", 1 << 17))
    reps = 6
    # one context per concurrent stream (a context's scratch is per call, include/b2f.h);
    # B2F_FILL_WGS is read only by the diagnostics build
    eng = b2f.Engine(0, diag=True)
    eng2 = b2f.Engine(0, diag=True)
    xa = synth.batch(n, rounds=12, seed=1)
    xb = synth.batch(n, rounds=12, seed=2)
    A, B = b2f.DeviceBatch(xa), b2f.DeviceBatch(xb)
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()
    for bt in (A, B):
        bt.fill(eng, s1.cuda_stream)
        bt.evaluate(eng, s1.cuda_stream)
    torch.cuda.synchronize()
    # back to back on one stream
    t0 = time.perf_counter()
    for k in range(reps):
        bt = A if k % 2 else B
        bt.fill(eng, s1.cuda_stream)
        bt.evaluate(eng, s1.cuda_stream)
    torch.cuda.synchronize()
    seq = (time.perf_counter() - t0) * 1e3 / reps
    # pipelined: fill(next) on s1 while eval(prev) on s2
    ev = [torch.cuda.Event() for _ in range(reps + 1)]
    A.fill(eng, s1.cuda_stream)
    ev[0].record(s1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(reps):
        cur, nxt = (A, B) if k % 2 == 0 else (B, A)
        s2.wait_event(ev[k])                 # cur filled
        cur.evaluate(eng2, s2.cuda_stream)
        done = torch.cuda.Event()
        done.record(s2)
        nxt.fill(eng, s1.cuda_stream)        # overlaps the eval above
        ev[k + 1].record(s1)
        s1.wait_event(done)                  # do not refill cur's buffers before its eval ended
    torch.cuda.synchronize()
    pipe = (time.perf_counter() - t0) * 1e3 / reps
    ok = A.report_dict()["first_failure"] == 2**64 - 1 and B.report_dict()["first_failure"] == 2**64 - 1
    print(json.dumps({"n": n, "fill_wgs": os.environ.get("B2F_FILL_WGS", "8"),
                      "sequential_ms_per_pair": round(seq, 3), "pipelined_ms_per_pair": round(pipe, 3),
                      "clean": ok}), flush=True)


if __name__ == "__main__":
    main()
