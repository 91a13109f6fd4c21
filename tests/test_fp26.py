"""The SM2 field in 10 x 26-bit limbs, Montgomery R = 2^286 (fp26.h), and the a = -3 point formulas on it
(ecp26.h), on the host: built with FE26_CHECK (every magnitude contract and limb bound asserted while the
cases run) and recomputed here with Python integers: Montgomery products mod p, k*G and the special
cases of madd/add in affine coordinates."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 2**256 - 2**224 - 2**96 + 2**64 - 1
N = 0xFFFFFFFEFFFFFFFFFFFFFFFFFFFFFFFF7203DF6B21C6052B53BBF40939D54123
A = P - 3
GX = 0x32C4AE2C1F1981195F9904466A39C9948FE30BBFF2660BE1715A4589334C74C7
GY = 0xBC3736A2F4F6779C59BDCEE36B692153D0A9877CC62A474002DF32E52139F0A0
R = 2**286
RINV = pow(R, -1, P)


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
        lam = (3 * p[0] * p[0] + A) * pow(2 * p[1], -1, P) % P
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


def _affine(X, Y, Z, inf):  # Montgomery coordinates
    if inf:
        return None
    X, Y, Z = X * RINV % P, Y * RINV % P, Z * RINV % P
    zi = pow(Z, -1, P)
    return X * zi * zi % P, Y * zi * zi * zi % P


@pytest.fixture(scope="module")
def lines(tmp_path_factory):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not found")
    exe = str(tmp_path_factory.mktemp("fp26") / "fp26_test")
    subprocess.run([cxx, "-O1", "-std=c++17", "-Wall", "-Wextra", "-Wno-unknown-pragmas", "-Werror",
                    "-o", exe, os.path.join(ROOT, "tests", "cpp", "fp26_test.cpp")], check=True)
    return subprocess.run([exe, "120"], check=True, capture_output=True, text=True).stdout.splitlines()


def test_field_ops_match_integers(lines):
    ops = {"mul": lambda a, b: a * b * RINV % P, "sqr": lambda a, b: a * a * RINV % P,
           "add": lambda a, b: (a + b) % P, "sub": lambda a, b: (a - b) % P, "neg": lambda a, b: -a % P,
           "norm": lambda a, b: a % P, "weak": lambda a, b: a % P}
    seen = dict.fromkeys(ops, 0)
    for ln in lines:
        f = ln.split()
        if f[0] != "F" or f[1] == "zchk":
            continue
        a, b, r = (_val(x) for x in f[2:5])
        assert r % P == ops[f[1]](a, b), ln
        if f[1] in ("mul", "sqr", "norm"):
            limbs = [int(x, 16) for x in f[4].split(",")]
            assert all(x <= 1 << 26 for x in limbs[:9]) and limbs[9] <= 1 << 22, ln  # magnitude 1
        if f[1] == "norm":
            assert r < P
        seen[f[1]] += 1
    assert all(v > 0 for v in seen.values()), seen


def test_is_zero(lines):
    n = 0
    for i, ln in enumerate(lines):
        f = ln.split()
        if f[0] != "Z":
            continue
        got, want = int(f[1]), int(f[2])
        if want == 2:
            want = int(_val(lines[i + 1].split()[2]) % P == 0)
        assert got == want, ln
        n += 1
    assert n > 100


def test_scalar_mult_by_double_and_madd(lines):
    g = (GX, GY)
    n = 0
    for ln in lines:
        f = ln.split()
        if f[0] == "P":
            assert _affine(_val(f[2]), _val(f[3]), _val(f[4]), f[5] == "1") == _mul(int(f[1], 16) % N, g), f[1]
            n += 1
    assert n == 20


def test_special_cases(lines):
    g = (GX, GY)
    want = {"madd_G": g, "madd_dbl": _mul(2, g), "madd_inf": None, "madd_from_inf": g, "add_6G": _mul(6, g),
            "add_dbl": _mul(2, g), "add_inf": None, "add_inf_l": _mul(4, g), "add_inf_r": _mul(4, g)}
    got = {}
    for ln in lines:
        f = ln.split()
        if f[0] == "A":
            got[f[1]] = _affine(_val(f[2]), _val(f[3]), _val(f[4]), f[5] == "1")
    assert got == want


def test_generated_asm_blocks_by_emulation():
    """fp26_mul_asm / fp26_sqr_asm (the device code of fp26_mul / fp26_sqr, generated into fe_asm.h) run
    instruction by instruction through tools/asm_emu.py on random and bound-hugging operands of magnitude
    1..15 (the contract's limit: column 8 reaches 2025 * 2^52 < 2^63): Montgomery products with
    magnitude-1 outputs."""
    import random
    import sys
    sys.path.insert(0, os.path.join(ROOT, "fisco-bcos_amd", "tools"))
    import asm_emu
    text = open(os.path.join(ROOT, "fisco-bcos_amd", "csrc", "fe_asm.h")).read()
    consts = {"k12": 1 << 12, "kn18": 0xFFFC0000, "kn16": 0xFFFF0000, "k22": 1 << 22}
    rng = random.Random(286)

    def val(l):
        return sum(x << (26 * i) for i, x in enumerate(l))

    for trial in range(120):
        m = rng.choice([1, 2, 4, 8, 11, 14, 15, 15])
        top = trial % 3 == 1

        def operand():
            if top:
                return [m << 26] * 9 + [m << 22]
            return [rng.randrange((m << 26) + 1) for _ in range(9)] + [rng.randrange((m << 22) + 1)]

        a, b = operand(), operand()
        vals = dict(consts, **{"a[%d]" % i: a[i] for i in range(10)}, **{"b[%d]" % i: b[i] for i in range(10)})
        for fn, want in (("fp26_mul_asm", val(a) * val(b) * RINV % P), ("fp26_sqr_asm", val(a) ** 2 * RINV % P)):
            out = asm_emu.run_block(text, fn, vals)
            r = [out["r[%d]" % i] for i in range(10)]
            assert val(r) % P == want, (fn, m, trial)
            assert all(x <= 1 << 26 for x in r[:9]) and r[9] <= 1 << 22, (fn, r)


def test_generator_is_on_the_curve():
    B = 0x28E9FA9E9D9F5E344D5A9E4BCF6509A7F39789F515AB8F92DDBCBD414D940E93
    assert (GY * GY - (GX**3 - 3 * GX + B)) % P == 0
