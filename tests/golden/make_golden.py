#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/.  Run in the build container only.

  kat.json          known-answer vectors transcribed from the reference's own tests (file:line cited)
  merkle.json       (a) roots the reference's own Merkle.h produced (compiled from
                        /root/reference in the survey container), (b) roots from an independent
                        pure-Python restatement (hashlib SM3 + the Keccak below) for more sizes,
                        cross-checked against (a) before being written
  ecc_openssl.json  secp256k1 recover / SM2 verify vectors computed by OpenSSL 1.1.1 EC
                        (oracle/xcheck_openssl.c; `make -C oracle xcheck` first)

Nothing here imports or runs reference code; the reference-produced values are data copied from
SURVEY.md.  The fixtures are data (inputs and expected outputs) only.
"""
import hashlib
import json
import os
import struct
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

# ---------------------------------------------------------------- pure-Python Keccak-256 (0x01 pad)
_RC = [0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
       0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
       0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
       0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
       0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
       0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008]
_ROT = [[0, 36, 3, 41, 18], [1, 44, 10, 45, 2], [62, 6, 43, 15, 61], [28, 55, 25, 21, 56],
        [27, 20, 39, 8, 14]]  # _ROT[x][y]
_M = (1 << 64) - 1


def _rol(v, r):
    return ((v << r) | (v >> (64 - r))) & _M if r else v


def _keccak_f(a):
    for rc in _RC:
        c = [a[x][0] ^ a[x][1] ^ a[x][2] ^ a[x][3] ^ a[x][4] for x in range(5)]
        d = [c[(x - 1) % 5] ^ _rol(c[(x + 1) % 5], 1) for x in range(5)]
        a = [[a[x][y] ^ d[x] for y in range(5)] for x in range(5)]
        b = [[0] * 5 for _ in range(5)]
        for x in range(5):
            for y in range(5):
                b[y][(2 * x + 3 * y) % 5] = _rol(a[x][y], _ROT[x][y])
        a = [[b[x][y] ^ ((~b[(x + 1) % 5][y]) & b[(x + 2) % 5][y]) for y in range(5)]
             for x in range(5)]
        a[0][0] ^= rc
    return a


def keccak256(msg: bytes) -> bytes:
    rate = 136
    m = bytearray(msg) + b"\x01"
    m += b"\x00" * ((-len(m)) % rate)
    m[-1] ^= 0x80
    a = [[0] * 5 for _ in range(5)]
    for off in range(0, len(m), rate):
        for i in range(rate // 8):
            a[i % 5][i // 5] ^= int.from_bytes(m[off + 8 * i: off + 8 * i + 8], "little")
        a = _keccak_f(a)
    return b"".join(a[i % 5][i // 5].to_bytes(8, "little") for i in range(4))


def sm3(msg: bytes) -> bytes:
    return hashlib.new("sm3", msg).digest()


HASHERS = {"keccak256": keccak256, "sm3": sm3}


# ------------------------------------------------------- Merkle restatements (Merkle.h / ParallelMerkleProof)
def merkle_new(h, width, leaves):
    """Merkle.h:170-208.  Returns the full output vector (count records as 32-B entries)."""
    if not leaves:
        raise ValueError("Empty input")
    if len(leaves) == 1:
        return [leaves[0]]
    out, level = [], leaves
    while len(level) > 1:
        nxt = [h(b"".join(level[i:i + width])) for i in range(0, len(level), width)]
        out.append(struct.pack(">I", len(nxt)) + b"\x00" * 28)
        out.extend(nxt)
        level = nxt
    return out


def merkle_old(h, leaves):
    """ParallelMerkleProof.cpp:32-69 (width 16, extra final hash, empty -> H(""))."""
    if not leaves:
        return h(b"")
    level = list(leaves)
    while len(level) > 1:
        level = [h(b"".join(level[i:i + 16])) for i in range(0, len(level), 16)]
    return h(level[0])


def bench_leaves(n):
    """merkleBench.cpp:18-34: leaf[i] = SM3(i as native (little-endian) size_t)."""
    return [sm3(struct.pack("<Q", i)) for i in range(n)]


# roots the reference's own Merkle.h produced (leaves = bench_leaves(n))
REFERENCE_ROOTS = {
    ("sm3", 16, 1): "b7869108f151ba70672e10153cc90fc2b5d4506a963f03b6c5b4aa3bcea09d83",
    ("sm3", 16, 2): "e18c79b7f2defdf1fd78690e6c47c8375ad61040b7973e6e75d0fdf1f6f4bb22",
    ("sm3", 16, 3): "b292daa166f99d6ea7f3ab124fda6dfe28eeb2f7187f7ebf4911a5e141183af0",
    ("sm3", 16, 17): "1f9ac75f82e1f0b6955634b2fc48b08ab48518d8e6716151c12345d73f6cecfe",
    ("sm3", 16, 100000): "585b83716f98127146c5a563e6905da9c6f26e54d5e0dd47f03bd2e8e4f149e7",
    ("keccak256", 2, 1): "b7869108f151ba70672e10153cc90fc2b5d4506a963f03b6c5b4aa3bcea09d83",
    ("keccak256", 2, 2): "5c8209a4fe35235393e51e18dd0694cd480db81a64c0062736a044e7f12be6f5",
    ("keccak256", 2, 3): "5ac4e47e19c5de07ed56e22c92e13efa1c0e838b4632d8460458c908a3a3feb7",
    ("keccak256", 2, 17): "741f553a7d060d82679d4dd31c12fc647d3871226808312d8807ace6d4ac5b50",
    ("keccak256", 2, 100000): "e334693ac00805161d751d7fabcb9ea111021e97d6dbddc7dfb278b075bc4e1d",
    ("keccak256", 16, 1): "b7869108f151ba70672e10153cc90fc2b5d4506a963f03b6c5b4aa3bcea09d83",
    ("keccak256", 16, 2): "5c8209a4fe35235393e51e18dd0694cd480db81a64c0062736a044e7f12be6f5",
    ("keccak256", 16, 3): "13684c6a18d4cc0cc6c4524756250268d59003c39367b6d369c21a561069b5f7",
    ("keccak256", 16, 17): "c6e1373321b1dd05c17df9012ac91e5c5eb5c4c214c6024955b6b6e49b88e964",
    ("keccak256", 16, 100000): "9eb6403797ecace0b94064597d58d7664402706836bc6f185324b0b73d03f526",
}
REFERENCE_OLD_SM3 = {1: "4f2c36a14bbea86f60efaeea213f87713ae502e9e521fe2b89ae85da4c99ecbf",
                     2: "f346019249b3d84eca6d5439859d94b6ad949ab5fc5c5e9b14df53ccee47a68b",
                     3: "388697a367de225cfc7c2164240c83fbe6792b282fcf3fd70aea1f9e4f7de658",
                     17: "a6268fdc43109a6c1100099fc1468d1b75e5a2eecb33818f55898045811193a5",
                     100000: "9af9068aad9b4efb45b924a396403937b77f5397361cbd84bf4d04060290d73d"}


def make_kat():
    kat = {
        "source": "transcribed from the reference's unit tests; see 'ref' per vector",
        "hash": [
            {"hasher": "keccak256", "msg": "", "digest": "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470", "ref": "bcos-crypto/test/unittests/HashTest.cpp:59-61"},
            {"hasher": "keccak256", "msg": "abcde", "digest": "6377c7e66081cb65e473c1b95db5195a27d04a7108b468890224bedbe1a8a6eb", "ref": "HashTest.cpp:63-67"},
            {"hasher": "keccak256", "msg": "hello", "digest": "1c8aff950685c2ed4bc3174f3472287b56d9517b9c948127319a09a7a36deac8", "ref": "HashTest.cpp:75-76"},
            {"hasher": "sm3", "msg": "", "digest": "1ab21d8355cfa17f8e61194831e81a8f22bec8c728fefb747ed035eb5082aa2b", "ref": "HashTest.cpp:82-84"},
            {"hasher": "sm3", "msg": "abcde", "digest": "afe4ccac5ab7d52bcae36373676215368baf52d3905e1fecbe369cc120e97628", "ref": "HashTest.cpp:86-89"},
            {"hasher": "sm3", "msg": "hello", "digest": "becbbfaae6548b8bf0cfcad5a27183cd1be6093b1cceccc303d9c61d0a645268", "ref": "HashTest.cpp:98-99"},
        ],
        "secp256k1_pubkey": [
            {"sk": "bcec428d5205abe0f0cc8a734083908d9eb8563e31f943d760786edf42ad67dd",
             "pub": "3378c2b7bcdce20357eb3dbb62590b88d4711dae74e1ea47dd4207441734d2fc7cf6df92fd8c0a3368ba5a1f5f9c3318d19a3f00ba2f2bd9f508b953be299fb5",
             "ref": "bcos-crypto/test/unittests/SignatureTest.cpp:53-63"}],
        "sm2_pubkey": [
            {"sk": "ca508b2b49c1d2dc46cbd5a011686fdc19937dbc704afe6c547a862b3e2b6c69",
             "pub": "f7dee65e76603ed7cd4c598d53cabe875c459e0fae4c6fd7b858189fd4741081e970bca0d5cb571a7ac30586aec71b23187d4b25e59143812f74a2744604d42b",
             "ref": "SignatureTest.cpp:238-243"}],
        "sm2_verify": [
            {"msg_hashed_with": "sm3", "msg": "abcd",
             "sig": "cd39bf939d999ca710576a629c962edfc28608701a3a7b61c971daeac5a1399cf4a7272fa80783e171c7fd5b038a3af4521f681ebe9fd44db3b60e750c438293f7dee65e76603ed7cd4c598d53cabe875c459e0fae4c6fd7b858189fd4741081e970bca0d5cb571a7ac30586aec71b23187d4b25e59143812f74a2744604d42b",
             "ok": True, "ref": "SignatureTest.cpp:238-251"}],
        "secp256k1_recover": [
            {"hash": "38d18acb67d25c8bb9942764b62f18e17054f66a817bd4295423adf9ed98873e",
             "sig": "38d18acb67d25c8bb9942764b62f18e17054f66a817bd4295423adf9ed98873e789d1dd423d25f0772d2748d60f7e4b81bb14d086eba8e8e8efb6dcff8a4ae0200",
             "ok": True, "address_keccak": "ceaccac640adf55b2028469bd36ba501f28b699d",
             "ref": "bcos-executor/test/old/EVMPrecompiledTest.cpp:58-72 (ecrecover, v=27 -> recid 0)"},
            {"hash": keccak256(b"abcd").hex(),
             "sig": keccak256(b"+++").hex() + keccak256(b"24324").hex() + "04",
             "ok": False, "ref": "SignatureTest.cpp:156-162 (v = 4 must throw InvalidSignature)"}],
    }
    return kat


def make_merkle():
    cases = []
    # (a) reference-produced roots, re-derived by the Python restatement as a cross-check
    for (hname, width, n), root in sorted(REFERENCE_ROOTS.items()):
        if hname == "keccak256" and n > 5000:
            got = root  # pure-Python Keccak too slow at 100k; this root stands on the reference alone
        else:
            got = merkle_new(HASHERS[hname], width, bench_leaves(n))[-1].hex()
        assert got == root, (hname, width, n, got, root)
        cases.append({"variant": "new", "hasher": hname, "width": width, "n": n, "root": root,
                      "source": "reference Merkle.h (SURVEY.md §8c)"})
    for n, root in sorted(REFERENCE_OLD_SM3.items()):
        assert merkle_old(sm3, bench_leaves(n)).hex() == root
        cases.append({"variant": "old", "hasher": "sm3", "width": 16, "n": n, "root": root,
                      "source": "restatement of ParallelMerkleProof.cpp:32-69 (SURVEY.md §8c)"})
    # (b) more sizes from the restatement (edges of every level boundary)
    sizes = [1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 33, 255, 256, 257, 1000, 4095, 4096, 4097]
    for hname in ("keccak256", "sm3"):
        for width in (2, 3, 4, 16):
            for n in sizes:
                if (hname, width, n) in REFERENCE_ROOTS:
                    continue
                if hname == "keccak256" and n > 1100 and width == 2:
                    continue
                tree = merkle_new(HASHERS[hname], width, bench_leaves(n))
                c = {"variant": "new", "hasher": hname, "width": width, "n": n,
                     "root": tree[-1].hex(), "source": "python restatement"}
                if n in (3, 17, 33):
                    c["tree"] = [e.hex() for e in tree]
                cases.append(c)
        for n in (0, 16, 257, 4097):
            if hname == "sm3" and n in REFERENCE_OLD_SM3:
                continue
            cases.append({"variant": "old", "hasher": hname, "width": 16, "n": n,
                          "root": merkle_old(HASHERS[hname], bench_leaves(n)).hex(),
                          "source": "python restatement"})
    for n in (20000, 100000):
        for width in (2, 16):
            if ("sm3", width, n) in REFERENCE_ROOTS:
                continue
            cases.append({"variant": "new", "hasher": "sm3", "width": width, "n": n,
                          "root": merkle_new(sm3, width, bench_leaves(n))[-1].hex(),
                          "source": "python restatement"})
    return {"leaves": "leaf[i] = SM3(le64(i)) (benchmark/merkleBench.cpp:18-34)",
            "tree_format": "per level: count record (uint32 BE + 28 zero bytes) then the level's nodes (Merkle.h:189-204)",
            "cases": cases}


def main():
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(make_kat(), f, indent=1)
    with open(os.path.join(HERE, "merkle.json"), "w") as f:
        json.dump(make_merkle(), f, indent=1)
    xc = os.path.join(HERE, "..", "..", "oracle", "_ref", "xcheck_openssl")
    if os.path.exists(xc):
        subprocess.run([xc, "400", os.path.join(HERE, "ecc_openssl.json")], check=True)
    else:
        print("oracle/_ref/xcheck_openssl not built; ecc_openssl.json left as is", file=sys.stderr)


if __name__ == "__main__":
    main()
