"""Static instruction counts of a gfx950 kernel's hot loop, from the compiler's assembly.

python tools/isa_count.py [KERNEL_SUBSTRING [SOURCE]]   (default: the 29-bit bucket chain
k_accumulate<false, true, 1> of csrc/msm.hip; e.g. `k_decide_wg decider.hip` for the decider)

Compiles snark-verifier-axiom_amd/csrc/msm.hip with hipcc -S (device only), takes the kernel's body,
and prints every basic block's instruction, v_mad_u64_u32 and VALU counts with its branch targets.
Which blocks form the per-entry common path has to be read off that control flow (the loop's
back edge, the rare branches it skips): for the round-6 29-bit chain the loop's common blocks hold
1,482 mads (madd_live's nine products, 1,467, plus address arithmetic), the doubling branch
(dbl_start) ~950 and the post-loop owner join (r29::add) ~2,280.  Rounds 4-5 identified the path
by a fixed rule (the doubling branch's lone 126-mad square), which no longer holds.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "snark-verifier-axiom_amd", "csrc", sys.argv[2] if len(sys.argv) > 2 else "msm.hip")
KEY = sys.argv[1] if len(sys.argv) > 1 else "k_accumulateILb0ELb1ELi1E"


def ops(lines):
    c = collections.Counter()
    for l in lines:
        s = l.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        c[s.split()[0]] += 1
    return c


def main():
    out = os.path.join(tempfile.mkdtemp(), "k.s")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                           "-S", "-o", out, SRC], stderr=subprocess.DEVNULL)
    text = open(out).read().split("\n")
    start = next(i for i, l in enumerate(text) if re.match(r"^_Z\S*%s\S*:" % KEY, l))
    end = next(i for i in range(start, len(text)) if text[i].startswith(".Lfunc_end"))
    body = text[start:end]
    # basic blocks
    blocks, cur, name = [], [], "entry"
    for l in body:
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            blocks.append((name, cur))
            cur, name = [], m.group(1)
        else:
            cur.append(l)
    blocks.append((name, cur))
    # the loop: from the first back-edge target to the last back-edge
    back = [i for i, (_, b) in enumerate(blocks) if any("s_branch" in l or "s_cbranch" in l for l in b)]
    total = ops(body)
    print("kernel %s: %d instructions, %d v_mad_u64_u32 (all paths, static)" % (KEY, sum(total.values()),
                                                                              total["v_mad_u64_u32"]))
    print("%-10s %6s %6s %6s  %s" % ("block", "instrs", "mads", "valu", "top opcodes"))
    for nm, b in blocks:
        c = ops(b)
        n = sum(c.values())
        if n == 0:
            continue
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        br = [l.split()[-1] for l in b if "branch" in l]
        print("%-10s %6d %6d %6d  %s  -> %s" % (nm, n, c["v_mad_u64_u32"], valu,
                                              ", ".join("%s %d" % kv for kv in c.most_common(4)), " ".join(br)))
    del back


if __name__ == "__main__":
    main()
