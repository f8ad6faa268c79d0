#!/usr/bin/env python3
"""Writes zfec_amd/csrc/gf_routines.inc: the multiply-by-constant routines of
matapply_bsr (kernels.hip) and the per-row calls into them.

GF(2^8) multiplication by c is linear over GF(2): on bit-planes p0..p7 of 32
bytes, output plane b of c*x is the XOR of the planes a whose bit b of c*2^a is
set (the same matrices as kernels.hip's make_bsg_bank and bitslice.cpp's
coef_masks).  With the fifteen XOR combinations L[m] of planes 0-3 and H[m] of
planes 4-7 in fixed registers, c*x added to an accumulator row is eight
v_xor3_b32 (acc_b ^= L[ml_b] ^ H[mh_b], the inline constant 0 for an empty
nibble).  Routine c holds exactly those eight instructions and returns; it sits
at zfec_gf_routines + 72*c (and at + 72*(256 + c) its "set" twin, which writes
c*x over the row instead of adding it: a wave's first input calls it, so no
accumulator is zeroed), so a kernel whose coefficients are run-time data
runs the instruction stream a specialised (JIT) kernel would have baked in, at
the cost of a call per coefficient instead of a compile per matrix.

Register contract (fixed by the routines' encodings):
  planes        p0..p7 at v8..v15: the single-plane combinations
  L[m], H[m]    the other eleven of each at v16..v26 / v27..v37
  accumulators  v[38 + b] + M0 index (the call sets gpr_idx(SRC0,DST) = 8 * row;
                row rr of a wave at v[38 + 8 rr .. 45 + 8 rr], rr < 10), last:
                a kernel with RT rows pins v8..v(37 + 8 RT); the block starts at
                v8, not higher, so RT = 10 (v8..v117) leaves the compiler ten
                registers below v128 and the kernel fits 4 waves per SIMD
                (round 5: bsr<10,lds> 144 -> 125 VGPRs, cfg4's first-seen
                20-row decode 0.498 -> 0.455 ms, profiles/r05_bsr_regs_ab.json)
  calls         s_swappc_b64 s[30:31] to the routine's absolute address, a 64-bit
                SGPR operand the kernel loads from its argument block or device-
                side table (the host writes zfec_gf_routines + 72 c there; it
                reads the table's address once per device, kernels.hip
                bsr_routine_base); the routine returns through s[30:31].  Round 4
                computed the address in the statement (s_getpc + the coefficient
                byte's extraction, multiply and 64-bit add: six scalar
                instructions per row against three now)
  M0            s_set_gpr_idx_on writes M0[7:0] and M0[15:12]; M0 is compiler-
                reserved (an "m0" clobber is ignored), so every bsr_input
                statement saves it into an early-clobber SGPR first and restores
                it last (s_nop 0 after the restore: an M0 write followed by an
                LDS-DMA / s_movrel needs one wait state)

Instruction forms (round 6).  On gfx950 a wave64 v_xor_b32 / v_mov_b32 issues
in half the cycles of any VOP3 instruction (v_bitop3_b32, shifts: 57-66 against
36-40 T lane-ops/s, profiles/r02_mb_valu.log), so a plane with one nibble
empty is `v_xor_b32 acc, acc, x` (VOP2: in gpr_idx(SRC0,DST) mode src0 is the
indexed accumulator, src1 the unindexed combination) and the "set" twins --
which ignore the row's old value -- are `v_xor_b32 acc, L, H` / `v_mov_b32 acc,
x`: their sources must not be indexed, so the first input's statement
(bsr_input_first / bsr_input_c_first) runs them in gpr_idx(DST) mode.
`--form legacy` writes round 5's routines (every plane a v_bitop3_b32, the set
twins in SRC0,DST mode) for the A/B (tools/ab_bsr.sh).

    python tools/gen_gf_routines.py            # rewrite the .inc
    python tools/gen_gf_routines.py --check    # exit 1 if it is stale
    python tools/gen_gf_routines.py --form legacy --out PATH
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "zfec_amd", "csrc", "gf_routines.inc")

ACC, PL, CB, STRIDE, MAX_ROWS = 38, 8, 16, 72, 10
MULTI = [m for m in range(1, 16) if m & (m - 1)]  # combinations that take XORs (11)


def reg(side, m):
    """Register of combination m (1..15) of planes 0-3 (side 0) or 4-7 (side 1)."""
    if m & (m - 1) == 0:
        return PL + 4 * side + (m.bit_length() - 1)
    return CB + 11 * side + MULTI.index(m)


def xtime(v):
    v <<= 1
    return (v ^ 0x11D) & 0xFF if v & 0x100 else v


def masks(c):
    p = [c]
    for _ in range(7):
        p.append(xtime(p[-1]))
    out = []
    for b in range(8):
        ml = sum(((p[a] >> b) & 1) << a for a in range(4))
        mh = sum(((p[a + 4] >> b) & 1) << a for a in range(4))
        out.append((ml, mh))
    return out


def routine(c, first=False, form="vop2", slot=0):
    """Routine c adds c*x to the accumulator row (acc_b ^= L ^ H); with
    first=True it sets the row to c*x instead (acc_b = L ^ H), so a wave's
    first input needs no zeroed accumulators.  form "legacy": every plane a
    v_bitop3_b32 (XOR3, truth table 0x96; the set twins 0x66, which ignores
    the row's old value, in SRC0,DST index mode).  form "vop2": XOR3 only
    where both nibbles are non-empty, VOP2 v_xor_b32 / VOP1 v_mov_b32 for the
    rest; the set twins run in DST-only index mode."""
    lines = []
    for b, (ml, mh) in enumerate(masks(c)):
        acc = ACC + 8 * slot + b  # slot: the row slot of the "slots" form (0 in the index-mode forms)
        if not ml and not mh and not first:
            continue
        sl = "v%d" % reg(0, ml) if ml else None
        sh = "v%d" % reg(1, mh) if mh else None
        if form == "legacy":  # (trunc64, slots: the vop2 instructions; trunc64 cut below)
            lines.append("v_bitop3_b32 v%d, v%d, %s, %s bitop3:%s" % (acc, acc, sl or "0", sh or "0",
                                                                     "0x66" if first else "0x96"))
        elif first:
            if sl and sh:
                lines.append("v_xor_b32 v%d, %s, %s" % (acc, sl, sh))
            else:
                lines.append("v_mov_b32 v%d, %s" % (acc, sl or sh or "0"))
        elif sl and sh:
            lines.append("v_bitop3_b32 v%d, v%d, %s, %s bitop3:0x96" % (acc, acc, sl, sh))
        else:
            lines.append("v_xor_b32 v%d, v%d, %s" % (acc, acc, sl or sh))
    if form == "trunc64":  # timing experiment only (wrong results): every routine cut to 64 bytes
        # (form "inline": the statements run one fixed routine's body in place of each call;
        # "noidx": the same without index mode, every row on row 0's registers)
        while routine_bytes(lines) + 4 > 64:
            lines.pop()
    lines.append("s_setpc_b64 s[30:31]")
    assert routine_bytes(lines) <= STRIDE
    return lines


def routine_bytes(lines):
    """Encoded size: VOP3 (v_bitop3_b32) 8 bytes, VOP1/VOP2 and SOP1 4."""
    return sum(8 if ln.startswith("v_bitop3") else 4 for ln in lines)


def statement(o, rt, cmb, first, form):
    """The asm statement of one input's calls for a wave of rt rows: cmb=False
    builds the 22 multi-plane combinations from the planes (bsr_input), cmb=True
    takes all 30 as inputs (bsr_input_c); first=True calls the set twins (the
    wave's first input), in DST-only index mode in the vop2 form."""
    mode = "gpr_idx(DST)" if first and form != "legacy" else "gpr_idx(SRC0,DST)"
    slots = form == "slots"
    o.append("    uint32_t keep;  // M0, saved and restored around the index-mode calls")
    o.append("    asm volatile(")
    if slots:  # no index mode: M0 untouched (keep stays an unused output)
        o.append("        \"; %%%d\\n\\t\"" % (8 * rt))
    else:
        o.append("        \"s_mov_b32 %%%d, m0\\n\\t\"" % (8 * rt))
    if not cmb:
        for side in (0, 1):
            for m in MULTI:
                top = 1 << (m.bit_length() - 1)
                o.append("        \"v_xor_b32 v%d, v%d, v%d\\n\\t\"" % (reg(side, m), reg(side, m ^ top), reg(side, top)))
    nout = 8 * rt
    nin = 8 if not cmb else 30
    for rr in range(rt):
        if form in ("noidx", "slots"):  # (noidx: a timing experiment only, wrong results)
            pass
        elif rr == 0:
            o.append("        \"s_set_gpr_idx_on 0, %s\\n\\t\"" % mode)
        elif form == "inlinefix":  # timing experiment only: index mode on, never moved (every row on row 0)
            pass
        else:
            o.append("        \"s_set_gpr_idx_idx %d\\n\\t\"" % (8 * rr))
        if form in ("inline", "noidx", "inlinefix"):  # timing experiments (wrong results): a fixed body, no call
            c = next(c for c in range(255, 0, -1) if all(ml and mh for ml, mh in masks(c)))
            for ln in routine(c, first=first, form="vop2")[:-1]:
                o.append("        \"%s\\n\\t\"" % ln)
            o.append("        \"s_nop 0 ; %%%d\\n\\t\"" % (nout + 1 + nin + rr))
            continue
        o.append("        \"s_swappc_b64 s[30:31], %%%d\\n\\t\"" % (nout + 1 + nin + rr))
    if form not in ("noidx", "slots"):
        o.append("        \"s_set_gpr_idx_off\\n\\t\"")
    if slots:
        o.append("        \"\"")
    else:
        o.append("        \"s_mov_b32 m0, %%%d\\n\\t\"" % nout)
        o.append("        \"s_nop 0\"")
    cons = "=" if first else "+"  # the set twins write every row they are called for
    outs = ['"%s{v%d}"(acc[%d][%d])' % (cons, ACC + 8 * rr + b, rr, b) for rr in range(rt) for b in range(8)]
    outs.append('"=&s"(keep)')
    if cmb:
        ins = ['"{v%d}"(q[%d])' % (PL + d, d) for d in range(30)]
    else:
        ins = ['"{v%d}"(p[%d])' % (PL + b, b) for b in range(8)]
    ins += ['"s"(addr[%d])' % rr for rr in range(rt)]
    clob = [] if cmb else ['"v%d"' % v for v in range(CB, CB + 22)]
    clob += ['"s30"', '"s31"', '"scc"']
    o.append("        : " + ", ".join(outs))
    o.append("        : " + ", ".join(ins))
    o.append("        : " + ", ".join(clob) + ");")


def render(form="vop2"):
    stride = 64 if form == "trunc64" else STRIDE
    o = []
    o.append("// gf_routines.inc -- generated by tools/gen_gf_routines.py; do not edit.")
    o.append("// The multiply-by-constant routines of matapply_bsr and the per-row calls")
    o.append("// into them (register contract and instruction forms in the generator's")
    o.append("// docstring).  Form: %s." % form)
    o.append("#pragma once")
    o.append("constexpr uint32_t kBsrStride = %d;   // bytes per routine" % stride)
    o.append("constexpr int kBsrMaxRows = %d;       // accumulator rows a wave can hold" % MAX_ROWS)
    o.append("constexpr uint32_t kBsrSetBase = %d;  // byte offset of the \"set\" routines (256 + c)" % (stride * 256))
    nslot = MAX_ROWS if form == "slots" else 1
    o.append("constexpr uint32_t kBsrSlotStride = %d;  // bytes per row slot's table (slots form; 0: index mode)"
             % (stride * 512 if nslot > 1 else 0))
    # clang drops file-scope asm from device compilations: the table is the body
    # of a device function nothing calls (kept by `used`; its label is a symbol
    # of the code object the kernels' calls resolve against)
    o.append("extern \"C\" __device__ __attribute__((noinline, used)) void zfec_gf_routine_table() {")
    # (a return, not a branch over the table: the slots form is past s_branch's +-128 KiB reach)
    o.append("asm volatile(\"s_setpc_b64 s[30:31]\\n\"")
    o.append("    \".p2align 6\\n\"")
    o.append("    \"zfec_gf_routines:\\n\"")
    for rr in range(nslot):
        for c in range(512):
            o.append("    \".org zfec_gf_routines + %d\\n\"" % (stride * (512 * rr + c)))
            o.append("    \"" + "\\n".join(routine(c % 256, first=c >= 256, form=form, slot=rr)) + "\\n\"")
    o.append("    \".org zfec_gf_routines + %d\\n\"" % (stride * 512 * nslot))
    o.append("    \"zfec_gf_routines_end:\\n\");")
    o.append("}")
    o.append("")
    o.append("// bsr_input<RT>(acc, p, addr): one input's contribution to a wave's RT rows.")
    o.append("// p = the input's eight bit-planes; addr[rr] = the absolute address of the")
    o.append("// routine of row rr's coefficient (zfec_gf_routines + 72 c, wave-uniform,")
    o.append("// written by the host).  Builds the 22 multi-plane combinations, then calls")
    o.append("// row rr's routine with the accumulator index at 8 * rr: index mode is set")
    o.append("// once and moved per row (s_set_gpr_idx_idx), so a row costs three scalar")
    o.append("// instructions (index, call, return).  bsr_input_first<RT>: the wave's first")
    o.append("// input, whose addresses are the set twins' (kBsrSetBase + 72 c).")
    for name, cmb, first in (("bsr_input", False, False), ("bsr_input_first", False, True),
                             ("bsr_input_c", True, False), ("bsr_input_c_first", True, True)):
        if name == "bsr_input_c":
            o.append("")
            o.append("// bsr_input_c<RT>(acc, q, addr): the same with the input's 30 combinations (planes")
            o.append("// and the 22 multi-plane XORs, in register order v%d..v%d) as inputs: built once per" % (PL, CB + 21))
            o.append("// workgroup and read from LDS by every wave (matapply_bsr's combination-sharing")
            o.append("// form), or built by the caller.")
        src = "const uint32_t (&q)[30]" if cmb else "const uint32_t (&p)[8]"
        o.append("template <int RT>")
        o.append("__device__ __forceinline__ void %s(uint32_t (&acc)[RT][8], %s, const uint64_t (&addr)[RT]);"
                 % (name, src))
        for rt in range(1, MAX_ROWS + 1):
            o.append("template <>")
            o.append("__device__ __forceinline__ void %s<%d>(uint32_t (&acc)[%d][8], %s, const uint64_t (&addr)[%d]) {"
                     % (name, rt, rt, src, rt))
            statement(o, rt, cmb, first, form)
            o.append("}")
    return "\n".join(o) + "\n"


def main():
    form = sys.argv[sys.argv.index("--form") + 1] if "--form" in sys.argv else "vop2"
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else OUT
    text = render(form)
    if "--check" in sys.argv:
        cur = open(out).read() if os.path.exists(out) else ""
        sys.exit(0 if cur == text else 1)
    with open(out, "w") as f:
        f.write(text)


if __name__ == "__main__":
    main()
