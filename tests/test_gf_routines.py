"""CPU checks of zfec_amd/csrc/gf_routines.inc, the multiply-by-constant
routines matapply_bsr calls (one per coefficient):

- the file is what tools/gen_gf_routines.py writes (no hand edits, no stale copy);
- every routine, executed by a small interpreter of its lines (v_bitop3_b32
  XOR3, VOP2 v_xor_b32, VOP1 v_mov_b32) on bit-planes of random bytes -- after
  the combination XORs that bsr_input emits -- adds exactly c * x (the
  oracle's gf_mul, zfec/fec.c:58-86 via oracle/fec_oracle.c) to the
  accumulator row, reading the row only where the index mode of its caller
  indexes it (SRC0 of the accumulate routines; the set twins' callers index
  the destination only);
- the "set" twins (256 + c) write c * x over the row;
- every routine fits its 72-byte slot (the .org directives would fail the
  build otherwise; this names the routine);
- the round-5 form (--form legacy) passes the same interpreter."""

import os
import re
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "zfec_amd", "csrc", "gf_routines.inc")
sys.path.insert(0, os.path.join(ROOT, "tools"))
from gen_gf_routines import ACC, PL  # noqa: E402  (the register contract)


def test_generated_file_is_current():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_gf_routines.py"), "--check"])
    assert r.returncode == 0, "gf_routines.inc differs from tools/gen_gf_routines.py output"


def _parse(text=None):
    text = text if text is not None else open(INC).read()
    body = text[text.index('"zfec_gf_routines:\\n"'):text.index('"zfec_gf_routines_end:')]
    routines = {}
    for m in re.finditer(r'"\.org zfec_gf_routines \+ (\d+)\\n"\s*\n\s*"([^"]*)"', body):
        routines[int(m.group(1))] = m.group(2).split("\\n")
    combos = re.search(r"bsr_input<1>.*?asm volatile\((.*?)s_swappc_b64", text, re.S).group(1)
    xors = re.findall(r"v_xor_b32 v(\d+), v(\d+), v(\d+)", combos)
    return routines, [(int(a), int(b), int(c)) for a, b, c in xors]


def _planes(x):
    """32 bytes -> 8 bit-planes (plane b: bit t = bit b of byte t)."""
    return [int(sum(((int(x[t]) >> b) & 1) << t for t in range(32))) for b in range(8)]


_OPS = [
    # (regex, kind): XOR3 of the accumulator (or, 0x66, of nothing) and two combinations
    (re.compile(r"v_bitop3_b32 v(\d+), v(\d+), (v\d+|0), (v\d+|0) bitop3:(0x96|0x66)"), "bitop3"),
    (re.compile(r"v_xor_b32 v(\d+), (v\d+), (v\d+)"), "xor"),
    (re.compile(r"v_mov_b32 v(\d+), (v\d+|0)"), "mov"),
]


def _bytes(line):
    return 8 if line.startswith("v_bitop3") else 4


def _check_routines(routines, xors, form):
    """Interpret every routine against the oracle.  Index-mode forms (legacy,
    vop2): 512 routines on row 0's registers (v38..v45), the caller's M0 index
    moving them to row rr.  The slots form: the 512 routines once per row slot
    rr (0..9), each on row rr's own registers v[38 + 8 rr ..], no index mode."""
    nslot = 10 if form == "slots" else 1
    assert len(routines) == 512 * nslot and len(xors) == 22
    rng = np.random.default_rng(72)
    mul = np.array([[oracle.gf_mul(a, b) for b in range(256)] for a in range(256)], dtype=np.uint8)
    for rr in range(nslot):
        acc_lo = ACC + 8 * rr
        rows = set(range(ACC, ACC + 80)) if form == "slots" else set(range(ACC, ACC + 8))
        for slot in range(512):
            c, first = slot % 256, slot >= 256
            lines = routines[72 * (512 * rr + slot)]
            assert lines[-2] == "s_setpc_b64 s[30:31]" and lines[-1] == "", (rr, slot, lines[-2:])
            body = lines[:-2]
            assert sum(_bytes(ln) for ln in body) + 4 <= 72, slot
            parsed = []
            for ln in body:
                for rx, kind in _OPS:
                    m = rx.fullmatch(ln)
                    if m:
                        parsed.append((kind, m.groups()))
                        break
                else:
                    raise AssertionError((slot, ln))
            if first:  # every plane written
                assert sorted(int(g[0]) for _, g in parsed) == list(range(acc_lo, acc_lo + 8)), (rr, slot)
            for trial in range(3 if rr == 0 else 1):
                x = rng.integers(0, 256, size=32, dtype=np.uint8)
                acc0 = rng.integers(0, 256, size=32, dtype=np.uint8)
                v = {}
                for b, pl in enumerate(_planes(x)):
                    v[PL + b] = pl
                for d, a, b in xors:
                    v[d] = v[a] ^ v[b]
                for b, pl in enumerate(_planes(acc0)):
                    v[acc_lo + b] = pl
                val = lambda s: 0 if s == "0" else v[int(s[1:])]
                # a row register is a source only as the routine's own row where the
                # caller's mode indexes it: SRC0 of the accumulate routines (legacy: of
                # the set twins too, whose 0x66 ignores it); never a set twin's source
                # in the vop2 and slots forms (no other row's register, ever)
                for kind, g in parsed:
                    d = int(g[0])
                    assert acc_lo <= d < acc_lo + 8, (rr, slot, kind, g)
                    if kind == "bitop3":
                        s0, s1, s2, tt = int(g[1]), g[2], g[3], g[4]
                        assert s0 == d, (slot, g)
                        assert tt == ("0x66" if first else "0x96"), (slot, g)
                        assert not (first and form != "legacy"), (slot, "set twins are VOP1/VOP2")
                        assert all(s == "0" or int(s[1:]) not in rows for s in (s1, s2)), (slot, g)
                        v[d] = (0 if first else v[s0]) ^ val(s1) ^ val(s2)
                    elif kind == "xor":
                        s0, s1 = g[1], g[2]
                        assert form != "legacy", (slot, g)
                        if first:  # sources: two combinations, none of them a row register
                            assert all(int(s[1:]) not in rows for s in (s0, s1)), (slot, g)
                            v[d] = val(s0) ^ val(s1)
                        else:  # src0 the routine's own row, src1 a combination
                            assert int(s0[1:]) == d and int(s1[1:]) not in rows, (slot, g)
                            v[d] = v[d] ^ val(s1)
                    else:
                        assert form != "legacy" and first, (slot, g)
                        assert g[1] == "0" or int(g[1][1:]) not in rows, (slot, g)
                        v[d] = val(g[1])
                want = _planes(mul[c][x] if first else acc0 ^ mul[c][x])
                assert [v[acc_lo + b] for b in range(8)] == want, (rr, slot, trial)


def _form(text):
    return re.search(r"Form: (\w+)\.", text).group(1)


def test_every_routine_multiplies():
    """Routines 0-255 add c * x to the row; 256-511 (the "set" twins a wave's
    first input calls) write c * x over whatever the row held (the shipped
    form, once per row slot in the slots form)."""
    text = open(INC).read()
    routines, xors = _parse(text)
    _check_routines(routines, xors, _form(text))


@pytest.mark.parametrize("form", ["legacy", "vop2", "slots"])
def test_generated_forms_multiply(tmp_path, form):
    """Every form tools/ab_build.sh can build (legacy: round 5's; vop2: round
    6's index-mode form; slots: one table per row slot, no index mode)."""
    out = tmp_path / (form + ".inc")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_gf_routines.py"), "--form", form, "--out",
                    str(out)], check=True)
    text = out.read_text()
    routines, xors = _parse(text)
    _check_routines(routines, xors, form)


def test_every_call_statement_restores_m0():
    """s_set_gpr_idx_on writes M0, which hipcc treats as reserved (an "m0"
    clobber is ignored: cdna_hip_programming.md, "Operands and clobbers"), so
    each bsr_input<RT> statement must save M0 into an early-clobber SGPR before
    its first index-mode call and restore it after its last one."""
    text = open(INC).read()
    bodies = re.findall(r"void (bsr_input(?:_c)?(?:_first)?)<(\d+)>\(.*?asm volatile\((.*?)\);\n\}", text, re.S)
    # bsr_input<1..10> (combinations built in the statement), bsr_input_first (the set
    # twins), bsr_input_c<1..10> (combinations as inputs), bsr_input_c_first
    assert [(fam, int(rt)) for fam, rt, _ in bodies] == [
        (fam, rt) for fam in ("bsr_input", "bsr_input_first", "bsr_input_c", "bsr_input_c_first") for rt in range(1, 11)]
    slots = _form(text) == "slots"
    for fam, rt, body in bodies:
        ins = [s for s in re.findall(r'"([^"]*)"', body.split("\n        :")[0])]
        ins = [ln.replace("\\n\\t", "") for ln in ins]
        if slots:  # no index mode: each row calls its own slot's routine, M0 is never written
            calls = [ln for ln in ins if ln.startswith("s_swappc_b64")]
            assert len(calls) == int(rt), (fam, rt)
            assert not any("m0" in ln or "gpr_idx" in ln for ln in ins), (fam, rt)
            continue
        save = [i for i, ln in enumerate(ins) if re.fullmatch(r"s_mov_b32 %(\d+), m0", ln)]
        restore = [i for i, ln in enumerate(ins) if re.fullmatch(r"s_mov_b32 m0, %(\d+)", ln)]
        idx_on = [i for i, ln in enumerate(ins) if ln.startswith("s_set_gpr_idx_on")]
        idx_idx = [i for i, ln in enumerate(ins) if ln.startswith("s_set_gpr_idx_idx")]
        idx_off = [i for i, ln in enumerate(ins) if ln.startswith("s_set_gpr_idx_off")]
        calls = [i for i, ln in enumerate(ins) if ln.startswith("s_swappc_b64")]
        # index mode on once, moved to row rr (8 rr) before each later call, off after the last
        assert len(idx_on) == 1 and len(idx_off) == 1 and len(calls) == int(rt), rt
        # the set twins run with only the destination indexed (their sources are
        # combinations); the accumulate routines index SRC0 (the row) and DST
        mode = "gpr_idx(DST)" if fam.endswith("_first") else "gpr_idx(SRC0,DST)"
        assert ins[idx_on[0]] == "s_set_gpr_idx_on 0, " + mode, (fam, rt, ins[idx_on[0]])
        assert [ins[i] for i in idx_idx] == ["s_set_gpr_idx_idx %d" % (8 * rr) for rr in range(1, int(rt))], rt
        assert idx_on[0] < calls[0] and calls[-1] < idx_off[0], rt
        assert all(calls[rr - 1] < idx_idx[rr - 1] < calls[rr] for rr in range(1, int(rt))), rt
        assert len(save) == 1 and len(restore) == 1, rt
        assert save[0] < idx_on[0] and restore[0] > idx_off[0], rt
        # no instruction after the restore writes M0, and the save and restore
        # name the same operand, which is an early-clobber SGPR output
        assert not any("m0" in ln or "gpr_idx_on" in ln for ln in ins[restore[0] + 1:]), rt
        n_save = re.fullmatch(r"s_mov_b32 %(\d+), m0", ins[save[0]]).group(1)
        n_rest = re.fullmatch(r"s_mov_b32 m0, %(\d+)", ins[restore[0]]).group(1)
        assert n_save == n_rest, rt
        outs = body.split("\n        :")[1]
        operands = re.findall(r'"([^"]+)"\(', outs)
        assert operands[int(n_save)] == "=&s", (rt, operands[int(n_save)])
