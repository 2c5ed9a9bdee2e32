"""Static ISA opcode histogram of a kernel, by issue-cost class (VERDICT r04/r05:
the mix of the fast table scorer's instructions).

    python tools/isa_histogram.py <device .s from hipcc --save-temps> <kernel substring> [out.json]

Counts every instruction of the kernel's function body (cold fallback code
included, so read it beside the dynamic per-class counts of tools/valu_mix.sh)
and, separately, the instructions of its innermost loop bodies (basic blocks
between a label and a backward branch to it), grouped as: quarter-rate
integer (32x32 multiplies: v_mad_u64_u32, v_mul_lo/hi_u32), transcendental
(v_exp/log/sqrt/rcp/rsq/sin/cos_f32), fp64, other 64-bit (shifts / adds on
register pairs), fp32 arithmetic, packed fp32 (v_pk_*_f32), 32-bit integer /
logic / compare / select, conversions, SALU, LDS, global memory, waits and
branches."""
import json
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("s_waitcnt") or op in ("s_nop", "s_barrier", "s_sleep"):
        return "wait"
    if op.startswith("s_cbranch") or op.startswith("s_branch") or op.startswith("s_setpc") or \
            op.startswith("s_endpgm"):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if not op.startswith("v_"):
        return "other"
    if op in ("v_mad_u64_u32", "v_mad_i64_i32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_hi_i32",
              "v_mul_lo_i32"):
        return "quarter_rate_int"
    if re.match(r"v_(exp|log|sqrt|rcp|rsq|sin|cos)(_legacy)?_f32", op):
        return "trans_f32"
    if op.endswith("_f64") or "_f64_" in op:
        return "fp64"
    if op.endswith(("_b64", "_u64", "_i64")) or "_u64_" in op or "_b64_" in op:
        return "int64"
    if op.startswith("v_pk_") and "f32" in op:
        return "pk_f32"
    if op.startswith("v_cvt"):
        return "cvt"
    if op.endswith(("_f32", "_f16")) or "_f32_" in op:
        return "fp32"
    return "int32_logic"


def kernel_body(lines, sub):
    start = None
    for i, ln in enumerate(lines):
        if start is None and re.match(r"^\S*%s\S*:" % re.escape(sub), ln) and "k_" in ln:
            start = i
        elif start is not None and ln.startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit("kernel %r not found" % sub)


def main(path, sub, out=None):
    lines = open(path).read().splitlines()
    body = kernel_body(lines, sub)
    insts = []  # (label index, opcode, operands)
    labels = {}
    for ln in body:
        s = ln.split(";")[0].strip()
        if not s or s.startswith("."):
            m = re.match(r"^(\.LBB\w+):", s)
            if m:
                labels[m.group(1)] = len(insts)
            continue
        if s.endswith(":"):
            continue
        op = s.split()[0]
        insts.append((op, s))
    total = Counter(classify(op) for op, _ in insts)
    # loop bodies: a branch at position j to a label at i <= j
    loops = []
    for j, (op, s) in enumerate(insts):
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            i = labels.get(tgt)
            if i is not None and i <= j:
                loops.append((i, j))
    inner = [(i, j) for i, j in loops
             if not any(a >= i and b <= j and (a, b) != (i, j) for a, b in loops)]
    loop_counts = []
    for i, j in sorted(inner, key=lambda x: x[1] - x[0], reverse=True)[:6]:
        c = Counter(classify(op) for op, _ in insts[i:j + 1])
        ops = Counter(op for op, _ in insts[i:j + 1])
        loop_counts.append({"first": i, "length": j - i + 1, "classes": dict(c),
                            "top_opcodes": dict(ops.most_common(12))})
    res = {"kernel": sub, "instructions": len(insts), "classes": dict(total.most_common()),
           "top_opcodes": dict(Counter(op for op, _ in insts).most_common(30)),
           "inner_loops": loop_counts}
    txt = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main(*sys.argv[1:])
