"""The SM2 lane-trio kernel's split of t P between its wave pairs (ecc_pair.hip, sm2_low_chain): waves
0 / 1 run Booth windows 63 .. split from digit 64 and then 4 split doublings, waves 2 / 3 run windows
split - 1 .. 0 from infinity on t shifted up by 4 (64 - split) bits.  Restated here on integers with the
kernel's digit rule (d = W + cb - 16 [W >= 8] from the top four bits W and the next bit cb) to show the
two sums add up to t for every split, and that the low chain's accumulator never meets the skipped
P = +-Q cases (|K| >= 16 before each addition of |d| <= 8, |K| < n).  CPU only."""
import random

N_SM2 = 0xFFFFFFFEFFFFFFFFFFFFFFFFFFFFFFFF7203DF6B21C6052B53BBF40939D54123
MASK = (1 << 256) - 1


def _windows(k, count):
    """`count` signed digits from the top of the 256-bit k, as the kernel's loop takes them (shl4)."""
    out = []
    for _ in range(count):
        W, cb = k >> 252, (k >> 251) & 1
        out.append(W + cb - 16 * (W >> 3))
        k = (k << 4) & MASK
    return out


def _high(t, split):
    acc = t >> 255  # digit 64 = bit 255
    for d in _windows(t, 64 - split):
        acc = 16 * acc + d
    return acc << (4 * split)


def _low(t, split):
    if split == 0:
        return 0
    ds = _windows((t << (4 * (64 - split))) & MASK, split)
    acc, first = 0, True
    for d in ds:
        if not first:
            acc *= 16
            assert acc == 0 or abs(acc) >= 16  # K P with |K| >= 16 (or infinity) before the addition
            assert acc == 0 or abs(acc) != abs(d)
        acc += d
        first = False
        assert abs(acc) < N_SM2
    return acc


def test_split_sums_to_t():
    rng = random.Random(5)
    edge = [0, 1, N_SM2 - 1, (1 << 255), (1 << 256) - 1, 0x8888888888888888 << 190, 0x7777777777777777 << 100]
    for t in edge + [rng.getrandbits(256) for _ in range(300)]:
        for split in (0, 1, 2, 16, 24, 32, 36, 38, 40, 63):
            assert _high(t, split) + _low(t, split) == t, (hex(t), split)
