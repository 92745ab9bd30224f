#!/usr/bin/env python3
"""Issue cost of VALU instruction kinds beside v_mfma_f32_16x16x4_f32 (timing probe, not part of
libdppo): cycles per MFMA slot of one wave per SIMD that issues NV instructions of a kind per MFMA
(mode 0), and of the VALU stream alone (mode 2), per instruction.

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/probe/mfma_probe.hip \\
        -o tools/probe/libmfma_probe.so
    python tools/probe/mfma_kind.py
"""
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
KINDS = ["v_fma_f32", "v_pk_fma_f32", "v_exp_f32", "v_add_f32", "v_pk_add_f32", "v_pk_mul_f32",
         "v_rcp_f32"]


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libmfma_probe.so"))
    lib.probe_mfma_kind.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 2 + [ctypes.c_int] * 2 + [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    blocks = torch.cuda.get_device_properties(dev).multi_processor_count
    out = torch.empty(blocks * 256, device=dev)
    cyc = torch.zeros(blocks * 8, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    iters = 4096
    for k, name in enumerate(KINDS):
        row = {"kind": name}
        for mode in (0, 2):
            for nv in (1, 2, 4, 8):
                for _ in range(2):
                    assert lib.probe_mfma_kind(k, nv, mode, out.data_ptr(), cyc.data_ptr(), iters,
                                               blocks, s) == 0
                torch.cuda.synchronize()
                c = float(cyc.view(blocks, 8)[:, :4].float().median()) / (iters * 16)
                if mode == 0:
                    row[f"mfma+{nv}"] = round(c, 2)
                else:
                    row[f"alone/ins@{nv}"] = round(c / nv, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
