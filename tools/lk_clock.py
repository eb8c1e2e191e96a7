"""Phase clocks of lk_zpass_kernel (diagnostics): runs the lookup columns of bench_lookup's
default workload on a variant library built with -DB2F_LK_CLOCK (tools/build_variant.sh) and
prints the s_memtime totals per phase, summed over waves, per call.
Usage: python3 tools/lk_clock.py zk-odst_amd/variants/libb2f_<name>.so"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zk-odst_amd"))

PHASES = {0: "ticket+samples", 1: "searches", 2: "den columns+suffix (+barrier)",
          3: "den scan + aggregate (den wave; others 0)", 4: "num columns+Q (+barrier)",
          10: "den wave: polls", 9: "den wave: after polls",
          5: "num scan / look-back (+barrier)", 6: "z"}


def main():
    import torch

    import b2f
    from b2f import synth

    lib = sys.argv[1]
    eng = b2f.Engine(0, lib_path=lib)
    batch = b2f.DeviceBatch(synth.batch(1 << 13, rounds=12))
    batch.fill(eng)
    s = torch.cuda.current_stream().cuda_stream
    eng.sync(s)
    usable = (1 << 17) - 7
    nc = min(64, batch.total_rows // usable)
    dev = batch.advice.device
    rb = torch.arange(nc, dtype=torch.int64, device=dev) * usable
    out = torch.empty((nc, 5, usable + 1, 4), dtype=torch.int64, device=dev)
    bad = torch.empty(nc, dtype=torch.int64, device=dev)
    th, be, ga = 0x1234567 << 200, 0x89abcdef << 180, 0x13579bdf << 190
    call = lambda: eng.lookup_columns_dev(batch.advice.data_ptr(), batch.total_rows,  # noqa
                                          rb.data_ptr(), nc, usable, th, be, ga, 1,
                                          out.data_ptr(), usable + 1, bad.data_ptr(), s)
    clk = ctypes.CDLL(lib).b2f_debug_lk_clock
    buf = (ctypes.c_uint64 * 24)()
    call()
    eng.sync(s)
    clk(buf)
    buf[13] = 0  # the reset value, the first start tick of the next calls
    reps = 3
    for _ in range(reps):
        call()
    eng.sync(s)
    clk(buf)
    tot = {PHASES[i]: round(buf[i] / reps / 1e6, 3) for i in PHASES}
    tot["max resident workgroups"] = buf[12]
    tot["polls per call"] = buf[15] / reps
    tot["blocks combined per call"] = buf[7] / reps
    tot["polls: block b+1 unpublished"] = buf[16] / reps
    tot["polls: a farther block unpublished"] = buf[17] / reps
    tot["reads: status before pieces"] = buf[18] / reps
    tot["span of the calls, 1e6 ticks"] = round((buf[14] - buf[13]) / 1e6, 3)
    print(json.dumps({"lib": lib, "unit": "1e6 s_memtime ticks per call, summed over waves", **tot}))


if __name__ == "__main__":
    main()
