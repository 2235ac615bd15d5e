"""Instruction mix of a kernel's loops from `hipcc -S` output: for each basic block range closed by a backward
branch (a loop), count MFMA, LDS reads/writes, transcendental and other VALU, SALU, waits and barriers.
  python tools/asm_loop_stats.py <file.s> <kernel symbol substring>"""
import re
import sys
from collections import Counter


def kernel_lines(path, sub):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(sub) + r"\S*:", l) or
                 (l.endswith(":") and sub in l and l.startswith("_Z")))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    return lines[start:end]


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "ds_read"
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "ds_write"
    if op.startswith("ds_"):
        return "ds_other"
    if op in ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32"):
        return "valu_trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    lines = kernel_lines(sys.argv[1], sys.argv[2])
    labels = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(lines):
        m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\d+_\d+)", l) or re.match(r"\s+s_branch\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            lo = labels[m.group(1)]
            c = Counter()
            for x in lines[lo:i + 1]:
                x = x.strip()
                if not x or x.startswith((";", ".")) or x.endswith(":"):
                    continue
                c[classify(x)] += 1
            print(f"loop {m.group(1)} lines {lo}-{i}: " + ", ".join(f"{k} {v}" for k, v in sorted(c.items())))
    vg = [l for l in lines if ".vgpr_count" in l or "NumVgprs" in l or "ScratchSize" in l or "Occupancy" in l]
    print("\n".join(v.strip() for v in vg[:6]))


if __name__ == "__main__":
    main()
