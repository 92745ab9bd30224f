#!/usr/bin/env python3
"""Co-issue of v_fma_f32 with v_mfma_f32_16x16x4_f32 on one SIMD (timing probe, not part of
libdppo): cycles per MFMA of a wave that issues NV independent FMAs per MFMA (mode 0, one wave per
SIMD), and of the same split over the two waves of a SIMD (mode 1).

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/probe/mfma_probe.hip \\
        -o tools/probe/libmfma_probe.so
    python tools/probe/mfma_valu.py
"""
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libmfma_probe.so"))
    lib.probe_mfma_valu.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    blocks = torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.empty(blocks * 512, device=dev)
    cyc = torch.zeros(blocks * 8, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    iters = 8192
    for mode in (0, 1):
        for nv in (0, 1, 2, 4, 6, 8):
            for _ in range(2):
                cyc.zero_()
                assert lib.probe_mfma_valu(nv, mode, out.data_ptr(), cyc.data_ptr(), iters, blocks,
                                           s) == 0
            torch.cuda.synchronize()
            c = cyc.view(blocks, 8).float()
            n = iters * 16
            print(json.dumps({"mode": mode, "valu_per_mfma": nv,
                              "mfma_wave_cycles_per_mfma": round(float(c[:, 0].median()) / n, 2),
                              "valu_wave_cycles_per_mfma": round(float(c[:, 4].median()) / n, 2)
                              if mode == 1 else None}), flush=True)


if __name__ == "__main__":
    main()
