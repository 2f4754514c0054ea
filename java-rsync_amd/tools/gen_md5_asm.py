"""Generates csrc/md5_asm.inc: the gfx950 MD5 compression used by the streaming block-sum kernel.

Why inline asm, and why in 7 blocks:
  * the compiler's own step puts a half-rate v_add3_u32 (a + m, F, K-from-SGPR) on the dependency chain;
    here every step is  F = v_bitop3(b, c, d);  t = X + F;  t = v_alignbit(t, t, 32 - s);  a = t + b
    with X = (m + K) + a formed off the chain by two full-rate VOP2 adds (K as a 32-bit literal);
  * the off-chain adds of step i+1 are placed between the chain instructions of step i, so a wave always
    has an independent instruction to issue while its chain op waits;
  * the backend puts an s_nop after every inline-asm statement (4 issue cycles each): one statement per
    step cost ~1 s_nop per step, so the 64 steps are grouped into 7 statements -- round 1 in four
    4-step pieces (each needs only the 4 words of one ds_read_b128, keeping the LDS waits interleaved),
    rounds 2, 3 and 4 whole.
Only plain VALU instructions (VOP2 add, bitop3, alignbit) appear: no software-managed hazards on gfx950.

usage: python gen_md5_asm.py > ../csrc/md5_asm.inc
"""

S = [7, 12, 17, 22] * 4 + [5, 9, 14, 20] * 4 + [4, 11, 16, 23] * 4 + [6, 10, 15, 21] * 4
K = [
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391,
]


def msg_index(i):
    if i < 16:
        return i
    if i < 32:
        return (5 * i + 1) % 16
    if i < 48:
        return (3 * i + 5) % 16
    return (7 * i) % 16


def bop(i):  # truth tables for (S0, S1, S2) = (b, c, d): F, G, H, I
    return ["0xca", "0xe4", "0x96", "0x39"][i // 16]


ROLES = [("a", "b", "c", "d"), ("d", "a", "b", "c"), ("c", "d", "a", "b"), ("b", "c", "d", "a")]
BLOCKS = [(0, 4), (4, 8), (8, 12), (12, 16), (16, 32), (32, 48), (48, 64)]


def block(lo, hi):
    lines = []
    words = sorted({msg_index(i) for i in range(lo, hi)} | ({msg_index(hi)} if hi < 64 else set()))
    for i in range(lo, hi):
        a, b, c, d = ROLES[i % 4]
        x_cur = "%[x0]" if i % 2 == 0 else "%[x1]"
        x_nxt = "%[x1]" if i % 2 == 0 else "%[x0]"
        lines.append(f"v_bitop3_b32 %[f], %[{b}], %[{c}], %[{d}] bitop3:{bop(i)}")
        if i + 1 < hi or hi < 64:
            lines.append(f"v_add_u32 %[y], 0x{K[i + 1]:08x}, %[m{msg_index(i + 1)}]")
        lines.append(f"v_add_u32 %[t], {x_cur}, %[f]")
        if i + 1 < hi or hi < 64:
            a_next = ROLES[(i + 1) % 4][0]
            lines.append(f"v_add_u32 {x_nxt}, %[y], %[{a_next}]")
        lines.append(f"v_alignbit_b32 %[t], %[t], %[t], {32 - S[i]}")
        lines.append(f"v_add_u32 %[{a}], %[t], %[{b}]")
    body = "\\n\\t".join(lines)
    ins = ", ".join(f'[m{w}] "v"(m[{w}])' for w in words)
    return (f'    asm("{body}"\n'
            f'        : [a] "+v"(a), [b] "+v"(b), [c] "+v"(c), [d] "+v"(d), [x0] "+v"(x0), [x1] "+v"(x1),\n'
            f'          [t] "=&v"(t), [f] "=&v"(f), [y] "=&v"(y)\n'
            f'        : {ins});')


def plain_block(lo, hi):
    """Steps lo..hi-1 in the per-step order: y = m + K; x = y + a; f = bitop3; t = x + f; rotate; a = t + b."""
    lines = []
    words = sorted({msg_index(i) for i in range(lo, hi)})
    for i in range(lo, hi):
        a, b, c, d = ROLES[i % 4]
        lines += [f"v_add_u32 %[t], 0x{K[i]:08x}, %[m{msg_index(i)}]",
                  f"v_add_u32 %[t], %[t], %[{a}]",
                  f"v_bitop3_b32 %[f], %[{b}], %[{c}], %[{d}] bitop3:{bop(i)}",
                  f"v_add_u32 %[t], %[t], %[f]",
                  f"v_alignbit_b32 %[t], %[t], %[t], {32 - S[i]}",
                  f"v_add_u32 %[{a}], %[t], %[{b}]"]
    body = "\\n\\t".join(lines)
    ins = ", ".join(f'[m{w}] "v"(m[{w}])' for w in words)
    return (f'    asm("{body}"\n'
            f'        : [a] "+v"(a), [b] "+v"(b), [c] "+v"(c), [d] "+v"(d), [t] "=&v"(t), [f] "=&v"(f)\n'
            f'        : {ins});')


def rot_block(lo, hi, nt, nop=False):
    """Plain per-step order with nt rotating (t, f) temporaries, so consecutive steps share no register."""
    lines = []
    words = sorted({msg_index(i) for i in range(lo, hi)})
    for i in range(lo, hi):
        a, b, c, d = ROLES[i % 4]
        t, f = f"%[t{i % nt}]", f"%[f{i % nt}]"
        lines += [f"v_add_u32 {t}, 0x{K[i]:08x}, %[m{msg_index(i)}]",
                  f"v_add_u32 {t}, {t}, %[{a}]",
                  f"v_bitop3_b32 {f}, %[{b}], %[{c}], %[{d}] bitop3:{bop(i)}",
                  f"v_add_u32 {t}, {t}, {f}",
                  f"v_alignbit_b32 {t}, {t}, {t}, {32 - S[i]}",
                  f"v_add_u32 %[{a}], {t}, %[{b}]"]
        if nop:
            lines.append("s_nop 0")
    body = "\\n\\t".join(lines)
    ins = ", ".join(f'[m{w}] "v"(m[{w}])' for w in words)
    tmps = ", ".join(f'[t{k}] "=&v"(t{k}), [f{k}] "=&v"(f{k})' for k in range(nt))
    return (f'    asm("{body}"\n'
            f'        : [a] "+v"(a), [b] "+v"(b), [c] "+v"(c), [d] "+v"(d), {tmps}\n'
            f'        : {ins});')


def main_rot(steps_per_block, nt, nop=False):
    out = [f"__device__ __forceinline__ void md5_compress_rot{steps_per_block}{'n' if nop else ''}(Md5State& st, const uint32_t (&m)[16]) {{",
           "    uint32_t a = st.a, b = st.b, c = st.c, d = st.d;",
           "    uint32_t " + ", ".join(f"t{k}, f{k}" for k in range(nt)) + ";"]
    for lo in range(0, 64, steps_per_block):
        out.append(rot_block(lo, lo + steps_per_block, nt, nop))
    out += ["    st.a += a;", "    st.b += b;", "    st.c += c;", "    st.d += d;", "}"]
    print("\n".join(out))


def main_plain(steps_per_block):
    out = [f"__device__ __forceinline__ void md5_compress_asm{steps_per_block}(Md5State& st, const uint32_t (&m)[16]) {{",
           "    uint32_t a = st.a, b = st.b, c = st.c, d = st.d, t, f;"]
    for lo in range(0, 64, steps_per_block):
        out.append(plain_block(lo, lo + steps_per_block))
    out += ["    st.a += a;", "    st.b += b;", "    st.c += c;", "    st.d += d;", "}"]
    print("\n".join(out))


def k3_block(lo, hi, nt):
    """rot16n with a + m + K as one v_add3_u32 (K from a VGPR: gfx950 VOP3 takes no literal), kbench A/B."""
    lines = []
    words = sorted({msg_index(i) for i in range(lo, hi)})
    for i in range(lo, hi):
        a, b, c, d = ROLES[i % 4]
        t, f = f"%[t{i % nt}]", f"%[f{i % nt}]"
        lines += [f"v_add3_u32 {t}, %[m{msg_index(i)}], %[{a}], %[k{i - lo}]",
                  f"v_bitop3_b32 {f}, %[{b}], %[{c}], %[{d}] bitop3:{bop(i)}",
                  f"v_add_u32 {t}, {t}, {f}",
                  f"v_alignbit_b32 {t}, {t}, {t}, {32 - S[i]}",
                  f"v_add_u32 %[{a}], {t}, %[{b}]",
                  "s_nop 0"]
    body = "\\n\\t".join(lines)
    ins = ", ".join([f'[m{w}] "v"(m[{w}])' for w in words] + [f'[k{i - lo}] "v"(kv[{i}])' for i in range(lo, hi)])
    tmps = ", ".join(f'[t{k}] "=&v"(t{k}), [f{k}] "=&v"(f{k})' for k in range(nt))
    return (f'    asm("{body}"\n'
            f'        : [a] "+v"(a), [b] "+v"(b), [c] "+v"(c), [d] "+v"(d), {tmps}\n'
            f'        : {ins});')


def main_k3(steps_per_block, nt):
    print("static constexpr uint32_t RSH_MD5_KTAB[64] = {" + ", ".join(f"0x{k:08x}u" for k in K) + "};")
    out = [f"__device__ __forceinline__ void md5_compress_k3_{steps_per_block}(Md5State& st, const uint32_t (&m)[16], const uint32_t (&kv)[64]) {{",
           "    uint32_t a = st.a, b = st.b, c = st.c, d = st.d;",
           "    uint32_t " + ", ".join(f"t{k}, f{k}" for k in range(nt)) + ";"]
    for lo in range(0, 64, steps_per_block):
        out.append(k3_block(lo, lo + steps_per_block, nt))
    out += ["    st.a += a;", "    st.b += b;", "    st.c += c;", "    st.d += d;", "}"]
    print("\n".join(out))


def k3s_block(lo, hi, nt, nop_every=1):
    """k3 with K from an SGPR operand (VOP3 takes one SGPR): a + m + K in one v_add3_u32 without the 64 VGPRs of
    constants; the compiler materialises each K with an s_mov_b32 (SALU, beside the other wave's VALU).  kbench A/B."""
    lines = []
    words = sorted({msg_index(i) for i in range(lo, hi)})
    for i in range(lo, hi):
        a, b, c, d = ROLES[i % 4]
        t, f = f"%[t{i % nt}]", f"%[f{i % nt}]"
        lines += [f"v_add3_u32 {t}, %[m{msg_index(i)}], %[{a}], %[k{i - lo}]",
                  f"v_bitop3_b32 {f}, %[{b}], %[{c}], %[{d}] bitop3:{bop(i)}",
                  f"v_add_u32 {t}, {t}, {f}",
                  f"v_alignbit_b32 {t}, {t}, {t}, {32 - S[i]}",
                  f"v_add_u32 %[{a}], {t}, %[{b}]"]
        if nop_every and (i + 1) % nop_every == 0:
            lines.append("s_nop 0")
    body = "\\n\\t".join(lines)
    ins = ", ".join([f'[m{w}] "v"(m[{w}])' for w in words] + [f'[k{i - lo}] "s"(0x{K[i]:08x}u)' for i in range(lo, hi)])
    tmps = ", ".join(f'[t{k}] "=&v"(t{k}), [f{k}] "=&v"(f{k})' for k in range(nt))
    return (f'    asm("{body}"\n'
            f'        : [a] "+v"(a), [b] "+v"(b), [c] "+v"(c), [d] "+v"(d), {tmps}\n'
            f'        : {ins});')


def main_k3s(steps_per_block, nt, nop_every=1, suffix=""):
    out = [f"__device__ __forceinline__ void md5_compress_k3s_{steps_per_block}{suffix}(Md5State& st, const uint32_t (&m)[16]) {{",
           "    uint32_t a = st.a, b = st.b, c = st.c, d = st.d;",
           "    uint32_t " + ", ".join(f"t{k}, f{k}" for k in range(nt)) + ";"]
    for lo in range(0, 64, steps_per_block):
        out.append(k3s_block(lo, lo + steps_per_block, nt, nop_every))
    out += ["    st.a += a;", "    st.b += b;", "    st.c += c;", "    st.d += d;", "}"]
    print("\n".join(out))


def main():
    out = ["// Generated by tools/gen_md5_asm.py -- do not edit.  See that script for the design.",
           "__device__ __forceinline__ void md5_compress_asm(Md5State& st, const uint32_t (&m)[16]) {",
           "    uint32_t a = st.a, b = st.b, c = st.c, d = st.d;",
           f"    uint32_t x0 = a + m[0] + 0x{K[0]:08x}u, x1 = 0, t, f, y;"]
    for lo, hi in BLOCKS:
        out.append(block(lo, hi))
    out += ["    st.a += a;", "    st.b += b;", "    st.c += c;", "    st.d += d;", "}"]
    print("\n".join(out))
    main_plain(4)
    main_plain(16)
    main_rot(4, 4)
    main_rot(16, 4)
    main_rot(4, 4, True)
    main_rot(16, 4, True)
    main_k3(8, 4)
    main_k3s(8, 4)
    main_k3s(16, 4)
    main_k3s(16, 4, 0, "_nonop")
    main_k3s(16, 4, 2, "_nop2")


if __name__ == "__main__":
    main()
