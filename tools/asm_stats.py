"""Per-kernel instruction mix of a hipcc -S listing (gfx950): MFMA, AGPR<->VGPR moves, VALU, LDS.

    python tools/asm_stats.py build.s [kernel-substring]
Static counts (instructions in the listing, not executed counts): a quick A/B of code shape.
"""
import re
import sys
from collections import Counter


def kernels(path):
    cur, out = None, {}
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m and not line.startswith("_Z") is False:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur and line.strip().startswith(".Lfunc_end"):
            cur = None
            continue
        if cur:
            s = line.strip()
            if s and not s.startswith((";", ".")) and not s.endswith(":"):
                out[cur].append(s.split()[0])
    return out


def main():
    ks = kernels(sys.argv[1])
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, ins in ks.items():
        if pat not in name:
            continue
        c = Counter(ins)
        mfma = sum(v for k, v in c.items() if k.startswith("v_mfma"))
        rd = c["v_accvgpr_read_b32"]
        wr = c["v_accvgpr_write_b32"]
        mv = c["v_accvgpr_mov_b32"]
        valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
        dsr = sum(v for k, v in c.items() if k.startswith("ds_read"))
        dsw = sum(v for k, v in c.items() if k.startswith("ds_write"))
        print(f"{name[:70]:70s} n={len(ins):6d} mfma={mfma:5d} acc_rd={rd:4d} acc_wr={wr:4d} "
              f"acc_mov={mv:3d} valu={valu:5d} ds_r={dsr:4d} ds_w={dsw:4d} "
              f"scratch={c['scratch_store_dword'] + c['scratch_load_dword']}")


if __name__ == "__main__":
    main()
