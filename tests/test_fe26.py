"""The 10 x 26-bit secp256k1 field and point formulas (fe26.h / ec26.h) on the host: built with
FE26_CHECK, so every magnitude contract and limb bound is asserted while the cases run, and every
result is recomputed here with Python integers (field ops mod p; k*G and the special cases of
madd/add in affine coordinates).  The same headers compile into the throughput kernels."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8


def _val(limbs):
    return sum(int(x, 16) << (26 * i) for i, x in enumerate(limbs.split(",")))


def _add(p, q):
    if p is None:
        return q
    if q is None:
        return p
    if p[0] == q[0] and (p[1] + q[1]) % P == 0:
        return None
    if p == q:
        lam = 3 * p[0] * p[0] * pow(2 * p[1], -1, P) % P
    else:
        lam = (q[1] - p[1]) * pow(q[0] - p[0], -1, P) % P
    x = (lam * lam - p[0] - q[0]) % P
    return x, (lam * (p[0] - x) - p[1]) % P


def _mul(k, pt):
    r = None
    for bit in bin(k)[2:]:
        r = _add(r, r)
        if bit == "1":
            r = _add(r, pt)
    return r


def _affine(X, Y, Z, inf):
    if inf:
        return None
    zi = pow(Z, -1, P)
    return X * zi * zi % P, Y * zi * zi * zi % P


@pytest.fixture(scope="module")
def lines(tmp_path_factory):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not found")
    exe = str(tmp_path_factory.mktemp("fe26") / "fe26_test")
    subprocess.run([cxx, "-O1", "-std=c++17", "-Wall", "-Wextra", "-Wno-unknown-pragmas", "-Werror",
                    "-o", exe, os.path.join(ROOT, "tests", "cpp", "fe26_test.cpp")], check=True)
    out = subprocess.run([exe, "150"], check=True, capture_output=True, text=True).stdout
    return out.splitlines()


def test_field_ops_match_integers(lines):
    ops = {"mul": lambda a, b: a * b % P, "sqr": lambda a, b: a * a % P, "add": lambda a, b: (a + b) % P,
           "sub": lambda a, b: (a - b) % P, "norm": lambda a, b: a % P, "weak": lambda a, b: a % P}
    seen = {k: 0 for k in list(ops) + ["sqrt"]}
    for ln in lines:
        f = ln.split()
        if f[0] != "F" or f[1] == "zchk":
            continue
        a, b, r = (_val(x) for x in f[2:5])
        if f[1] == "sqrt":
            assert r * r % P == a, ln
            assert r < P
        else:
            assert r % P == ops[f[1]](a, b), ln
        if f[1] == "norm":
            assert r < P and all(int(x, 16) < (1 << 26) for x in f[4].split(",")), ln
        seen[f[1]] += 1
    assert all(v > 0 for v in seen.values()), seen


def test_is_zero(lines):
    checked = 0
    for i, ln in enumerate(lines):
        f = ln.split()
        if f[0] != "Z":
            continue
        got, want = int(f[1]), int(f[2])
        if want == 2:
            nxt = lines[i + 1].split()
            assert nxt[1] == "zchk"
            want = int(_val(nxt[2]) % P == 0)
        assert got == want, ln
        checked += 1
    assert checked > 100


def test_scalar_mult_by_double_and_madd(lines):
    g = (GX, GY)
    n = 0
    for ln in lines:
        f = ln.split()
        if f[0] != "P":
            continue
        k = int(f[1], 16)
        got = _affine(_val(f[2]), _val(f[3]), _val(f[4]), f[5] == "1")
        assert got == _mul(k % N, g), f[1]
        n += 1
    assert n == 24


def test_special_cases(lines):
    g = (GX, GY)
    want = {"madd_3G": _mul(3, g), "madd_dbl": _mul(2, g), "madd_inf": None, "madd_from_inf": g,
            "add_6G": _mul(6, g), "add_dbl": _mul(2, g), "add_inf": None, "add_inf_l": _mul(4, g),
            "add_inf_r": _mul(4, g)}
    got = {}
    for ln in lines:
        f = ln.split()
        if f[0] == "A":
            got[f[1]] = _affine(_val(f[2]), _val(f[3]), _val(f[4]), f[5] == "1")
    assert got == want


def test_generated_asm_blocks_by_emulation():
    """fe26_mul_asm / fe26_sqr_asm, the device code of fe26_mul / fe26_sqr (fe_asm.h, generated), run
    instruction by instruction through tools/asm_emu.py on random and bound-hugging operands of
    magnitude 1..16; the emulator also rejects operand forms the hardware does not take (a
    v_lshl_add_u64 shift above 4)."""
    import random
    import sys
    sys.path.insert(0, os.path.join(ROOT, "fisco-bcos_amd", "tools"))
    import asm_emu
    text = open(os.path.join(ROOT, "fisco-bcos_amd", "csrc", "fe_asm.h")).read()
    consts = {"kR0": 0x3D10, "k1024": 1024, "kR0x": 0x3D10 << 10, "k20": 1 << 20, "k977": 977}
    rng = random.Random(26)

    def val(l):
        return sum(x << (26 * i) for i, x in enumerate(l))

    for trial in range(120):
        m = rng.choice([1, 2, 4, 8, 16])
        top = trial % 3 == 1

        def operand():
            if top:
                return [m << 26] * 9 + [m << 22]
            return [rng.randrange((m << 26) + 1) for _ in range(9)] + [rng.randrange((m << 22) + 1)]

        a, b = operand(), operand()
        vals = dict(consts, **{"a[%d]" % i: a[i] for i in range(10)}, **{"b[%d]" % i: b[i] for i in range(10)})
        for fn, want in (("fe26_mul_asm", val(a) * val(b) % P), ("fe26_sqr_asm", val(a) ** 2 % P)):
            out = asm_emu.run_block(text, fn, vals)
            r = [out["r[%d]" % i] for i in range(10)]
            assert val(r) % P == want, (fn, m, trial)
            assert all(x <= 1 << 26 for x in r[:9]) and r[9] <= 1 << 22, (fn, r)  # magnitude 1
