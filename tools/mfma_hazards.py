"""Wait-state audit of the inline-asm MFMAs in a hipcc -S listing (gfx950).

    python tools/mfma_hazards.py build/mbwave.s [kernel-substring]

LLVM's hazard recognizer does not see an MFMA written as inline asm (`mfma4_acc` in
csrc/mbwave.hip), so the wait states around it are checked here, on the listing of every kernel
instantiation, by a forward data-flow pass over the kernel's basic blocks (loop back-edges
included; at a join the shortest distance wins):

  R1  VALU write of a VGPR/AGPR -> asm MFMA reading it (SrcA/B/C)            >= 2 states
  R2  asm MFMA write of its D    -> any other instruction reading or writing
      those registers (v_accvgpr_read/mov, VALU, stores, a compiler MFMA),
      except the next asm MFMA taking the same tuple whole as SrcC          >= 12 states
      (16x16x4 f32 = 8-pass XDL; gfx950 adds one state to gfx940's 11)
  R3  asm MFMA reading SrcC      -> a non-MFMA instruction writing it (WAR)  >= 11 states

and, for the packed-fp32 VALU steps written as inline asm (csrc/mbwave.hip `pk_*`), which the
recognizer does not see either:

  R4  asm VALU write             -> a compiler MFMA reading it (SrcA/B/C)    >= 2 states
  R5  transcendental VALU write  -> asm VALU reading it                      >= 2 states
      (v_exp / v_rcp / v_log / v_sqrt / v_rsq / v_sin / v_cos; gfx940 needs 1)
  R6  compiler MFMA write of D   -> asm VALU reading or writing those regs   >= 12 states
  R7  compiler MFMA reading SrcC -> asm VALU writing it (WAR)                >= 11 states
  R8  asm VALU write             -> a DPP / permlane instruction reading it  >= 2 states

A state is one issued instruction (`s_nop N` = N + 1).  An MFMA's own issue counts as one.  The
count is conservative where the listing is ambiguous (an instruction's first vector operand is
taken as written and every operand as read).  Exit status 1 and one line per violation if any.
"""
from __future__ import annotations

import re
import sys

R1, R2, R3 = 2, 12, 11
R4, R5, R6, R7, R8 = 2, 2, 12, 11, 2
TRANS = ("v_exp_f32", "v_rcp_f32", "v_log_f32", "v_sqrt_f32", "v_rsq_f32", "v_sin_f32",
         "v_cos_f32", "v_rcp_iflag_f32")
CAP = 16
REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")
BRANCH = re.compile(r"^s_(branch|cbranch_\w+)$")


def regs(op: str):
    out = []
    for m in REG.finditer(op):
        k = m.group(1)
        if m.group(4) is not None:
            out.append(f"{k}{m.group(4)}")
        else:
            out += [f"{k}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)]
    return out


def parse(path, pat=""):
    """{kernel: [(kind, text, ...)]}: kind 'label' / 'ins'; instructions keep an asm flag."""
    kernels, cur, in_asm = {}, None, False
    for line in open(path):
        s = line.strip()
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1) if pat in m.group(1) else None
            if cur:
                kernels[cur] = []
            continue
        if cur is None:
            continue
        if s.startswith(".Lfunc_end"):
            cur = None
            continue
        if s == ";;#ASMSTART":
            in_asm = True
            continue
        if s == ";;#ASMEND":
            in_asm = False
            continue
        s = s.split(";")[0].strip()      # trailing comments (";  =>This Inner Loop Header")
        if not s:
            continue
        if s.endswith(":") and not s.startswith("s_"):
            kernels[cur].append(("label", s[:-1]))
            continue
        if s.startswith("."):
            continue
        kernels[cur].append(("ins", s, in_asm))
    return kernels


def states(ins: str) -> int:
    m = re.match(r"^s_nop\s+(\d+)", ins)
    return int(m.group(1)) + 1 if m else 1


def decode(ins: str):
    """(mnemonic, written regs, read regs, srcC regs or None)."""
    parts = ins.split(None, 1)
    op = parts[0]
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    allr = [r for o in ops for r in regs(o)]
    if op.startswith("v_mfma"):
        d = regs(ops[0])
        return op, d, [r for o in ops[1:] for r in regs(o)], regs(ops[3]) if len(ops) > 3 else []
    if op.startswith(("global_store", "buffer_store", "ds_write", "scratch_store", "flat_store",
                      "ds_store")):
        return op, [], allr, None
    w = regs(ops[0]) if ops else []
    if op.startswith(("v_permlane", "v_swap")) and len(ops) > 1:
        w = w + regs(ops[1])
    return op, w, allr, None


def check(kernel, items):
    # basic blocks
    blocks, cur, labels = [], [], {}
    for it in items:
        if it[0] == "label":
            if cur:
                blocks.append(cur)
            cur = []
            labels[it[1]] = len(blocks)
            blocks.append(None)   # placeholder: the label starts the next block
            continue
        cur.append(it)
        op = it[1].split()[0]
        if BRANCH.match(op) or op == "s_endpgm" or op == "s_setpc_b64":
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    # resolve placeholders: label index -> index of the next real block
    real, label_block = [], {}
    for i, b in enumerate(blocks):
        if b is None:
            continue
        real.append(b)
    idx = -1
    remap = {}
    for i, b in enumerate(blocks):
        if b is not None:
            idx += 1
        else:
            remap[i] = idx + 1
    for name, i in labels.items():
        label_block[name] = remap[i]
    succ = []
    for bi, b in enumerate(real):
        last = b[-1][1].split()
        op = last[0]
        s = []
        if BRANCH.match(op):
            tgt = last[1] if len(last) > 1 else None
            if tgt in label_block:
                s.append(label_block[tgt])
            if op != "s_branch" and bi + 1 < len(real):
                s.append(bi + 1)
        elif op not in ("s_endpgm", "s_setpc_b64") and bi + 1 < len(real):
            s.append(bi + 1)
        succ.append(s)
    # state: reg -> distance (states since) for: valu write, asm-mfma write (+ tuple), asm-mfma
    # srcC read, asm-valu write, transcendental write, compiler-mfma write, compiler-mfma srcC read
    empty = ({}, {}, {}, {}, {}, {}, {})
    ins_state = [None] * len(real)
    ins_state[0] = empty
    work = [0]
    viol = set()

    def age(st, n):
        return tuple({k: (min(CAP, v[0] + n),) + v[1:] for k, v in d.items()} for d in st)

    def merge(a, b):
        out = []
        for da, db in zip(a, b):
            d = dict(da)
            for k, v in db.items():
                if k not in d or v[0] < d[k][0]:
                    d[k] = v
            out.append(d)
        return tuple(out)

    while work:
        bi = work.pop()
        st = ins_state[bi]
        vw, mw, cr, aw, tw, cmw, ccr = (dict(x) for x in st)
        for n, it in enumerate(real[bi]):
            text, is_asm = it[1], it[2]
            op, w, r, srcc = decode(text)
            is_mfma = op.startswith("v_mfma")
            is_avalu = is_asm and op.startswith("v_") and not is_mfma
            if is_mfma and not is_asm:
                for x in r:
                    if x in aw and aw[x][0] < R4:
                        viol.add(("R4", kernel, text, x, aw[x][0]))
            if is_avalu:
                for x in r:
                    if x in tw and tw[x][0] < R5:
                        viol.add(("R5", kernel, text, x, tw[x][0]))
                for x in set(r) | set(w):
                    if x in cmw and cmw[x][0] < R6:
                        viol.add(("R6", kernel, text, x, cmw[x][0]))
                for x in w:
                    if x in ccr and ccr[x][0] < R7:
                        viol.add(("R7", kernel, text, x, ccr[x][0]))
            if ("dpp" in text or "quad_perm" in text or "row_" in text or
                    op.startswith("v_permlane")) and not is_asm:
                for x in r:
                    if x in aw and aw[x][0] < R8:
                        viol.add(("R8", kernel, text, x, aw[x][0]))
            if is_asm and is_mfma:
                for x in r:
                    if x in vw and vw[x][0] < R1:
                        viol.add(("R1", kernel, text, x, vw[x][0]))
                    if x in mw and mw[x][0] < R2 and not (x in srcc and mw[x][1] == tuple(srcc)):
                        viol.add(("R2", kernel, text, x, mw[x][0]))
            else:
                for x in set(r) | set(w):
                    if x in mw and mw[x][0] < R2:
                        viol.add(("R2", kernel, text, x, mw[x][0]))
                if not is_mfma:
                    for x in w:
                        if x in cr and cr[x][0] < R3:
                            viol.add(("R3", kernel, text, x, cr[x][0]))
            k = states(text)
            # age everything by this instruction's states, then apply its effects
            for d in (vw, mw, cr, aw, tw, cmw, ccr):
                for x in list(d):
                    v = d[x]
                    nv = min(CAP, v[0] + k)
                    if nv >= CAP:
                        del d[x]
                    else:
                        d[x] = (nv,) + v[1:]
            if is_mfma:
                for x in w:
                    vw.pop(x, None)
                    aw.pop(x, None)
                    tw.pop(x, None)
                    if is_asm:
                        mw[x] = (0, tuple(w))
                        cmw.pop(x, None)
                    else:
                        mw.pop(x, None)
                        cmw[x] = (0,)
                for x in srcc:
                    if is_asm:
                        cr[x] = (0,)
                    else:
                        ccr[x] = (0,)
            elif op.startswith("v_"):
                for x in w:
                    vw[x] = (0,)
                    mw.pop(x, None)
                    cmw.pop(x, None)
                    if is_asm:
                        aw[x] = (0,)
                    else:
                        aw.pop(x, None)
                    if op.split("_e32")[0].split("_e64")[0] in TRANS:
                        tw[x] = (0,)
                    else:
                        tw.pop(x, None)
            else:
                for x in w:     # loads: no VALU hazard, but they end an MFMA result's life
                    for d in (vw, aw, tw, cmw):
                        d.pop(x, None)
        out = (vw, mw, cr, aw, tw, cmw, ccr)
        for sb in succ[bi]:
            new = out if ins_state[sb] is None else merge(ins_state[sb], out)
            if new != ins_state[sb]:
                ins_state[sb] = new
                work.append(sb)
    return sorted(viol)


def main(argv):
    path = argv[1]
    pat = argv[2] if len(argv) > 2 else ""
    ks = parse(path, pat)
    total = 0
    n_asm = 0
    for k, items in ks.items():
        n_asm += sum(1 for it in items if it[0] == "ins" and it[2] and it[1].startswith("v_mfma"))
        v = check(k, items)
        total += len(v)
        for rule, kern, text, reg, dist in v:
            print(f"{rule} {kern[:60]} `{text}` {reg}: {dist} states")
    print(f"{len(ks)} kernels, {n_asm} asm MFMAs, {total} violations")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
