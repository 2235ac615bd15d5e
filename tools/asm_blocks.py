"""Per-basic-block instruction classes of one kernel in `hipcc -S` output (loop blocks marked by the compiler's
'in Loop' comments): python tools/asm_blocks.py <file.s> <kernel symbol substring> [--ops LABEL ...]"""
import collections
import re
import sys


def main():
    path, sub = sys.argv[1], sys.argv[2]
    want = sys.argv[sys.argv.index("--ops") + 1:] if "--ops" in sys.argv else []
    L = open(path).read().split("\n")
    s = next(i for i, l in enumerate(L) if re.match(r"^_Z\S*" + re.escape(sub) + r"\S*:", l))
    e = next(i for i in range(s, len(L)) if L[i].strip().startswith(".Lfunc_end"))
    cur, cnt, ops = "entry", collections.Counter(), collections.Counter()
    out = []
    for x in L[s + 1:e] + [".LBBend:"]:
        t = x.strip()
        m = re.match(r"^(\.LBB\d+_\d+|\.LBBend):(.*)", t)
        if m:
            out.append((cur, dict(cnt), ops))
            cur, cnt, ops = m.group(1) + (" loop" if "Loop" in m.group(2) else ""), collections.Counter(), collections.Counter()
            continue
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        ops[op] += 1
        k = ("mfma" if op.startswith("v_mfma") else "trans" if op in ("v_exp_f32_e32", "v_log_f32_e32", "v_rcp_f32_e32")
             else "ds" if op.startswith("ds_") else "valu" if op.startswith("v_") else "vmem"
             if op.startswith(("global_", "buffer_")) else "salu")
        cnt[k] += 1
    for name, c, o in out:
        if sum(c.values()):
            print(name, c)
            if any(name.startswith(w) for w in want):
                print("   ", sorted(o.items(), key=lambda kv: -kv[1]))


if __name__ == "__main__":
    main()
