"""GPU field arithmetic (FieldK1, fe.h / fe_asm.h) against Python integers, including the rare
carry/borrow tails of the branch-over-tail k1_add/k1_sub asm (word-1 overflow, second fold) that random
inputs essentially never reach.  Runs fisco-bcos_amd/lib/fetest (built by `make -C fisco-bcos_amd`)."""
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "fisco-bcos_amd", "lib", "fetest")
P = 2**256 - 2**32 - 977
C = 2**32 + 977
M = 2**256


def _cases():
    rnd = random.Random(5)
    edge = [0, 1, 2, C - 1, C, C + 1, P - 1, P, P + 1, M - 1, M - 2, M - C, M - C - 1, M - C + 1,
            2**64 - C, 2**64 - C - 1, 2**64 - 1, 2**63, 2**255, 2**224 - 1]
    cases = []
    for a in edge:
        for b in edge:
            for op in ("add", "sub", "mul"):
                cases.append((op, a, b))
        cases.append(("sqr", a, 0))
        cases.append(("norm", a, 0))
    # add: low two words of a + b - 2^256 just below 2^64 - c (word-1 carry, first-fold tail)
    for _ in range(300):
        s = (rnd.randrange(M) >> 64 << 64) | (2**64 - 1 - rnd.randrange(C))
        a = rnd.randrange(s + 1, M)
        cases.append(("add", a, s + M - a))
        t = rnd.randrange(0, C)          # sub: a - b + 2^256 = t < c forces the borrow tail
        b = rnd.randrange(t + 1, M)
        cases.append(("sub", t + M - b, b))
    # shifted passes: 2^k a and 3a for a in [0, 2^256); the top bits shifted out fold back, and
    # 2^k a close to a multiple of 2^256 (low two words near 2^64 - fold) drives the carry tail
    for a in edge:
        for op in ("shl1", "shl2", "shl3", "mul3"):
            cases.append((op, a, 0))
    for _ in range(300):
        k = rnd.choice((1, 2, 3))
        hi = rnd.randrange(2**k)
        low = (rnd.randrange(M) >> 64 << 64) | (2**64 - 1 - rnd.randrange(C * (2**k)))
        a = ((hi << 256) | low) >> k           # 2^k a = hi * 2^256 + low (up to the shifted-out bits)
        cases.append(("shl%d" % k, a, 0))
        cases.append(("mul3", rnd.randrange(M - 2**70, M), 0))
        hi = rnd.randrange(1, 2**k)      # 2^k a = hi * 2^256 + (2^256 - small): the second fold
        cases.append(("shl%d" % k, ((hi << 256) | (M - 1 - rnd.randrange(C * hi))) >> k, 0))
    for _ in range(500):
        cases.append((rnd.choice(("add", "sub", "mul", "sqr", "shl1", "shl2", "shl3", "mul3")),
                      rnd.randrange(M), rnd.randrange(M)))
    return cases


@pytest.mark.gpu
def test_fieldk1_vs_python():
    assert os.path.exists(EXE), "build fisco-bcos_amd/lib/fetest first (make -C fisco-bcos_amd)"
    cases = _cases()
    text = "\n".join("%s %x %x" % c for c in cases) + "\n"
    r = subprocess.run([EXE], input=text, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = [int(x, 16) for x in r.stdout.split()]
    assert len(got) == len(cases)
    for (op, a, b), g in zip(cases, got):
        want = {"add": a + b, "sub": a - b, "mul": a * b, "sqr": a * a, "norm": a, "shl1": 2 * a,
                "shl2": 4 * a, "shl3": 8 * a, "mul3": 3 * a}[op] % P
        assert g == want, (op, hex(a), hex(b), hex(g), hex(want))
