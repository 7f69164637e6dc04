"""Instruction mix of a kernel's basic blocks from its gfx950 assembly
(profiling aid for the issue-cycle floor of a wave role).

  hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \\
        --cuda-device-only -S or-gym-inventory_amd/csrc/newsvendor.hip -o /tmp/nv.s
  python tools/isa_mix.py /tmp/nv.s nv_roll_kernelILi5ELb0ENS_3Pcg [--rates profiles/r04/valu_rates.txt]

Prints, per basic block: instruction count by class (quarter-rate 32/64-bit
integer multiplies, f64, other VALU, SALU, LDS, VMEM, waits), the loop it
closes (back-edge), and its VALU issue cycles per wave with the measured
per-instruction issue intervals (tools/valu_rates), 4 cycles for an op not
measured.  Blocks are in layout order, not execution order.
"""
import argparse
import collections
import re

CLASSES = ("mad64", "mul32", "f64", "trans", "valu", "salu", "lds", "vmem", "wait")


def classify(op):
    if op.startswith("v_mad_u64_u32") or op.startswith("v_mad_i64_i32"):
        return "mad64"
    if op.startswith("v_mul_lo_u32") or op.startswith("v_mul_hi_u32") or op.startswith("v_mul_hi_i32"):
        return "mul32"
    if op.startswith(("v_rcp_", "v_rsq_", "v_sqrt_", "v_log_", "v_exp_", "v_sin_", "v_cos_")):
        return "trans"
    if re.match(r"v_\w+_f64", op) or op.startswith("v_div_") or op.startswith("v_ldexp_f64") \
            or op.startswith("v_frexp_") and "f64" in op:
        return "f64"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "salu"


def load_rates(path):
    """cycles per wave-instruction at W = 1 from tools/valu_rates output"""
    rates = {}
    if not path:
        return rates
    for line in open(path):
        m = re.match(r"(\S+)\s+W=1\s+([\d.]+) cycles/instr", line)
        if m:
            rates[m.group(1)] = float(m.group(2))
    return rates


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("symbol", help="substring of the kernel's mangled name")
    ap.add_argument("--rates", default=None)
    args = ap.parse_args()
    rates = load_rates(args.rates)
    lines = open(args.asm).read().split("\n")
    start = next(i for i, l in enumerate(lines) if args.symbol in l and l.endswith(":") is False
                 and re.match(r"^_Z\S+:", l) and args.symbol in l.split(":")[0])
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    print(lines[start].split(":")[0])
    blocks, cur = [], ["entry", []]
    for l in lines[start + 1:end]:
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            blocks.append(cur)
            cur = [m.group(1), []]
            continue
        t = l.strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        cur[1].append(t.split(";")[0].strip())
    blocks.append(cur)
    idx = {b[0]: i for i, b in enumerate(blocks)}
    tot = collections.Counter()
    for i, (name, ins) in enumerate(blocks):
        c = collections.Counter(classify(x.split()[0]) for x in ins)
        tot.update(c)
        cyc = 0.0
        for x in ins:
            op = x.split()[0]
            k = classify(op)
            if k in ("salu", "wait", "lds", "vmem"):
                continue
            base = re.sub(r"_e(32|64)$", "", op)
            cyc += rates.get(base, 16.0 if k in ("mad64", "mul32", "trans") else 4.0)
        back = [b.split()[-1] for b in ins if b.startswith(("s_cbranch", "s_branch"))
                and b.split()[-1] in idx and idx[b.split()[-1]] <= i]
        tag = "  loop<-" + ",".join(back) if back else ""
        print(f"{i:3d} {name:14s} n={len(ins):4d} valu_cyc={cyc:7.0f} "
              + " ".join(f"{k}={c[k]}" for k in CLASSES if c[k]) + tag)
    print("total " + " ".join(f"{k}={tot[k]}" for k in CLASSES if tot[k]))


if __name__ == "__main__":
    main()
