#!/usr/bin/env python3
"""Cycles per v_mfma_f32_16x16x4_f32 for 1/2/4 accumulator chains per wave, with 1 or 2 waves per
SIMD (timing probe, not part of libdppo).

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/probe/mfma_probe.hip \
        -o tools/probe/libmfma_probe.so
    python tools/probe/mfma_probe.py
"""
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libmfma_probe.so"))
    lib.probe_mfma.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                               ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    blocks = torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.empty(blocks * 512, device=dev)
    cyc = torch.zeros(blocks * 8 + 16, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    iters = 4096
    for nacc in (1, 2, 4):
        for waves in (4, 8):
            for _ in range(2):
                cyc.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert lib.probe_mfma(nacc, out.data_ptr(), cyc.data_ptr(), iters, waves, waves,
                                      blocks, s) == 0
                e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            tflops = blocks * waves * iters * 8 * nacc * 2048 / (ms * 1e-3) / 1e12
            c = cyc[:blocks * 8].view(blocks, 8)[:, :waves].float()
            ab = cyc[blocks * 8:].view(8, 2).cpu().numpy()
            ab = (ab - ab[0, 0])[:waves].tolist()
            n = iters * 8 * nacc
            print(json.dumps({"acc_chains": nacc, "waves_per_simd": waves // 4,
                              "cycles_per_mfma_per_wave": round(float(c.median()) / n, 2),
                              "simd_cycles_per_mfma": round(float(c.median()) / n / (waves // 4), 2),
                              "kernel_ms": round(ms, 4), "tflops": round(tflops, 1),
                              "memtime_ghz": round(float(c.median()) / (ms * 1e6), 3), "block0_t0_t1": ab}),
                  flush=True)


if __name__ == "__main__":
    main()
