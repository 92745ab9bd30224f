"""Static count of s_waitcnt forms per mbw_kernel instantiation in a hipcc -S listing (A/B of
code shape; not a timing):  python tools/isa_waits.py a.s [b.s]"""
import collections
import re
import sys


def counts(path):
    out, cur = {}, None
    for line in open(path):
        m = re.match(r"^(_Z\S*mbw_kernel\S*):", line)
        if m:
            cur = m.group(1)
            out[cur] = collections.Counter()
            continue
        if cur and line.startswith(".Lfunc_end"):
            cur = None
        if cur:
            s = line.strip().split(";")[0]
            if s.startswith("s_waitcnt"):
                out[cur][s] += 1
            elif s.startswith(("ds_read", "v_mfma", "v_readlane", "v_writelane")):
                out[cur][s.split()[0].split("_e")[0]] += 1
    return out


if __name__ == "__main__":
    res = [counts(p) for p in sys.argv[1:]]
    for k in res[0]:
        name = re.search(r"kernelILi(\d)ELb(\d)ELi(\d)ELb(\d)", k).groups()
        row = []
        for r in res:
            c = r.get(k, collections.Counter())
            row.append(f"lgkm0={c['s_waitcnt lgkmcnt(0)']:4d} vm0={c['s_waitcnt vmcnt(0)']:3d} "
                       f"dsr={sum(v for kk, v in c.items() if kk.startswith('ds_read')):4d} "
                       f"rdl={c['v_readlane_b32']:3d} wrl={c['v_writelane_b32']:3d}")
        print("A%s C%s NIB%s X%s | " % name + " | ".join(row))
