"""Generate tools/experimental/bs_sbox.inc: the AES S-box as a bitsliced Boolean circuit for gfx950.

The circuit is the 115-gate (83 XOR/XNOR + 32 AND) Boyar-Peralta S-box network (published in
"A new combinational logic minimization technique with applications to cryptology", SEA 2010).
It is restated here as data and checked against the FIPS-197 S-box on all 256 inputs before
anything is written. Gates whose result feeds exactly one other gate are then folded into that
gate whenever the combination still has at most three distinct inputs: gfx950's v_bitop3_b32
evaluates any 3-input truth table in one VALU op. The folded network is re-checked on all 256
inputs, and emitted as straight-line device code over 32-bit bit planes (bit k of every plane =
block k), so one call evaluates 32 S-boxes per lane.

Run: python3 tools/gen_bs_sbox.py   (writes the .inc; prints gate counts)
"""
import itertools
import os
import sys

SBOX = bytes.fromhex(
    "637c777bf26b6fc53001672bfed7ab76ca82c97dfa5947f0add4a2af9ca472c0"
    "b7fd9326363ff7cc34a5e5f171d8311504c723c31896059a071280e2eb27b275"
    "09832c1a1b6e5aa0523bd6b329e32f8453d100ed20fcb15b6acbbe394a4c58cf"
    "d0efaafb434d338545f9027f503c9fa851a3408f929d38f5bcb6da2110fff3d2"
    "cd0c13ec5f974417c4a77e3d645d197360814fdc222a908846eeb814de5e0bdb"
    "e0323a0a4906245cc2d3ac629195e479e7c8376d8dd54ea96c56f4ea657aae08"
    "ba78252e1ca6b4c6e8dd741f4bbd8b8a703eb5664803f60e613557b986c11d9e"
    "e1f8981169d98e949b1e87e9ce5528df8ca1890dbfe6426841992d0fb054bb16")

# (out, op, a, b): op in "^" (xor), "&" (and), "^~" (xnor: a ^ ~b). Inputs x0 (MSB) .. x7 (LSB),
# outputs s0 (MSB) .. s7 (LSB).
GATES = """
y14 x3 ^ x5; y13 x0 ^ x6; y9 x0 ^ x3; y8 x0 ^ x5; t0 x1 ^ x2; y1 t0 ^ x7; y4 y1 ^ x3;
y12 y13 ^ y14; y2 y1 ^ x0; y5 y1 ^ x6; y3 y5 ^ y8; t1 x4 ^ y12; y15 t1 ^ x5; y20 t1 ^ x1;
y6 y15 ^ x7; y10 y15 ^ t0; y11 y20 ^ y9; y7 x7 ^ y11; y17 y10 ^ y11; y19 y10 ^ y8;
y16 t0 ^ y11; y21 y13 ^ y16; y18 x0 ^ y16;
t2 y12 & y15; t3 y3 & y6; t4 t3 ^ t2; t5 y4 & x7; t6 t5 ^ t2; t7 y13 & y16; t8 y5 & y1;
t9 t8 ^ t7; t10 y2 & y7; t11 t10 ^ t7; t12 y9 & y11; t13 y14 & y17; t14 t13 ^ t12;
t15 y8 & y10; t16 t15 ^ t12; t17 t4 ^ t14; t18 t6 ^ t16; t19 t9 ^ t14; t20 t11 ^ t16;
t21 t17 ^ y20; t22 t18 ^ y19; t23 t19 ^ y21; t24 t20 ^ y18;
t25 t21 ^ t22; t26 t21 & t23; t27 t24 ^ t26; t28 t25 & t27; t29 t28 ^ t22; t30 t23 ^ t24;
t31 t22 ^ t26; t32 t31 & t30; t33 t32 ^ t24; t34 t23 ^ t33; t35 t27 ^ t33; t36 t24 & t35;
t37 t36 ^ t34; t38 t27 ^ t36; t39 t29 & t38; t40 t25 ^ t39;
t41 t40 ^ t37; t42 t29 ^ t33; t43 t29 ^ t40; t44 t33 ^ t37; t45 t42 ^ t41;
z0 t44 & y15; z1 t37 & y6; z2 t33 & x7; z3 t43 & y16; z4 t40 & y1; z5 t29 & y7;
z6 t42 & y11; z7 t45 & y17; z8 t41 & y10; z9 t44 & y12; z10 t37 & y3; z11 t33 & y4;
z12 t43 & y13; z13 t40 & y5; z14 t29 & y2; z15 t42 & y9; z16 t45 & y14; z17 t41 & y8;
t46 z15 ^ z16; t47 z10 ^ z11; t48 z5 ^ z13; t49 z9 ^ z10; t50 z2 ^ z12; t51 z2 ^ z5;
t52 z7 ^ z8; t53 z0 ^ z3; t54 z6 ^ z7; t55 z16 ^ z17; t56 z12 ^ t48; t57 t50 ^ t53;
t58 z4 ^ t46; t59 z3 ^ t54; t60 t46 ^ t57; t61 z14 ^ t57; t62 t52 ^ t58; t63 t49 ^ t58;
t64 z4 ^ t59; t65 t61 ^ t62; t66 z1 ^ t63; s0 t59 ^ t63; s6 t56 ^~ t62; s7 t48 ^~ t60;
t67 t64 ^ t65; s3 t53 ^ t66; s4 t51 ^ t66; s5 t47 ^ t65; s1 t64 ^~ s3; s2 t55 ^~ t67
"""

OUTS = [f"s{i}" for i in range(8)]
INS = [f"x{i}" for i in range(8)]


def parse():
    gates = []
    for item in GATES.replace("\n", " ").split(";"):
        f = item.split()
        if not f:
            continue
        out, a, op, b = f
        gates.append((out, op, a, b))
    return gates


def tt_of(op):
    # 2-input truth table over (a, b), index = a*2 + b
    return {"^": [0, 1, 1, 0], "&": [0, 0, 0, 1], "^~": [1, 0, 0, 1]}[op]


def to_nodes(gates):
    """node: out -> (inputs tuple, truth table dict {assignment tuple: bit})"""
    nodes = {}
    for out, op, a, b in gates:
        t = tt_of(op)
        nodes[out] = ((a, b), {(x, y): t[2 * x + y] for x in (0, 1) for y in (0, 1)})
    return nodes


def evaluate(nodes, order, x):
    env = {f"x{i}": (x >> (7 - i)) & 1 for i in range(8)}
    for n in order:
        ins, tt = nodes[n]
        env[n] = tt[tuple(env[i] for i in ins)]
    return sum(env[f"s{i}"] << (7 - i) for i in range(8))


def check(nodes, order, what):
    for x in range(256):
        if evaluate(nodes, order, x) != SBOX[x]:
            sys.exit(f"{what}: mismatch at input {x:#04x}")


def fold(nodes, order):
    """Fold single-use nodes into their consumer while the consumer keeps <= 3 inputs."""
    changed = True
    while changed:
        changed = False
        uses = {n: [] for n in nodes}
        for n in order:
            for i in nodes[n][0]:
                if i in uses:
                    uses[i].append(n)
        for g in order:
            if g in OUTS or len(uses[g]) != 1:
                continue
            h = uses[g][0]
            gin, gtt = nodes[g]
            hin, htt = nodes[h]
            new_in = tuple(dict.fromkeys([i for i in hin if i != g] + list(gin)))
            if len(new_in) > 3:
                continue
            new_tt = {}
            for asg in itertools.product((0, 1), repeat=len(new_in)):
                env = dict(zip(new_in, asg))
                env[g] = gtt[tuple(env[i] for i in gin)]
                new_tt[asg] = htt[tuple(env[i] for i in hin)]
            nodes[h] = (new_in, new_tt)
            del nodes[g]
            order.remove(g)
            changed = True
            break
    return nodes, order


def bitop3_code(ins, tt):
    """v_bitop3 operands and immediate for a node: bit idx of the immediate is the output for
    (S0, S1, S2) = (idx >> 2 & 1, idx >> 1 & 1, idx & 1) (S0 = 0xF0, S1 = 0xCC, S2 = 0xAA). A
    2-input node repeats its last input; indices that would need the repeat to differ never occur."""
    ops = list(ins) + [ins[-1]] * (3 - len(ins))
    code = 0
    for idx in range(8):
        vals = ((idx >> 2) & 1, (idx >> 1) & 1, idx & 1)
        env, ok = {}, True
        for name, v in zip(ops, vals):
            if name in env and env[name] != v:
                ok = False
            env[name] = v
        if ok and tt[tuple(env[n] for n in ins)]:
            code |= 1 << idx
    return ops, code


def emit(nodes, order):
    lines = []
    n_ops = 0
    for n in order:
        ins, tt = nodes[n]
        if len(ins) == 2:
            a, b = ins
            t = [tt[(0, 0)], tt[(0, 1)], tt[(1, 0)], tt[(1, 1)]]
            if t == [0, 1, 1, 0]:
                expr = f"{a} ^ {b}"
            elif t == [0, 0, 0, 1]:
                expr = f"{a} & {b}"
            elif t == [1, 0, 0, 1]:
                expr = f"~({a} ^ {b})"
            else:
                ops, code = bitop3_code(ins, tt)
                expr = f"bs_op3<{code:#04x}>({ops[0]}, {ops[1]}, {ops[2]})"
        else:
            ops, code = bitop3_code(ins, tt)
            expr = f"bs_op3<{code:#04x}>({ops[0]}, {ops[1]}, {ops[2]})"
        lines.append(f"    const uint32_t {n} = {expr};")
        n_ops += 1
    return lines, n_ops


def main():
    gates = parse()
    nodes = to_nodes(gates)
    order = [g[0] for g in gates]
    check(nodes, order, "Boyar-Peralta circuit")
    n0 = len(order)
    nodes, order = fold(nodes, order)
    check(nodes, order, "folded circuit")
    lines, n_ops = emit(nodes, order)
    # re-check the emitted 3-input codes by evaluating them bitwise
    env_nodes = {}
    for n in order:
        ins, tt = nodes[n]
        ops, code = bitop3_code(ins, tt)
        env_nodes[n] = (ops, code)
    for x in range(256):
        env = {f"x{i}": (x >> (7 - i)) & 1 for i in range(8)}
        for n in order:
            ops, code = env_nodes[n]
            idx = env[ops[0]] * 4 + env[ops[1]] * 2 + env[ops[2]]
            env[n] = (code >> idx) & 1
        if sum(env[f"s{i}"] << (7 - i) for i in range(8)) != SBOX[x]:
            sys.exit(f"emitted bitop3 codes: mismatch at {x:#04x}")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "tools", "experimental", "bs_sbox.inc")
    with open(out, "w") as f:
        f.write("// GENERATED by tools/gen_bs_sbox.py — do not edit. The Boyar-Peralta AES S-box circuit\n")
        f.write(f"// ({n0} gates) folded to {n_ops} ops of at most 3 inputs (v_bitop3_b32), checked on all\n")
        f.write("// 256 inputs by the generator. p[7] = MSB plane ... p[0] = LSB plane; in place.\n")
        f.write("__device__ __forceinline__ void bs_sbox(uint32_t (&p)[8]) {\n")
        for i in range(8):
            f.write(f"    const uint32_t x{i} = p[{7 - i}];\n")
        f.write("\n".join(lines) + "\n")
        for i in range(8):
            f.write(f"    p[{7 - i}] = s{i};\n")
        f.write("}\n")
    print(f"gates {n0} -> ops {n_ops}; wrote {out}")


if __name__ == "__main__":
    main()
