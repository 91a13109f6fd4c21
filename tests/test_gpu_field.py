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
    for _ in range(500):
        cases.append((rnd.choice(("add", "sub", "mul", "sqr")), rnd.randrange(M), rnd.randrange(M)))
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
        want = {"add": a + b, "sub": a - b, "mul": a * b, "sqr": a * a, "norm": a}[op] % P
        assert g == want, (op, hex(a), hex(b), hex(g), hex(want))
