"""Per-round latencies of the small-batch kernel variants from a tools/small_sweep.py line (tx mode),
relative to the lane-trio kernel's round: the `lat` table of ecc_txv.hip auto_kernel (and bench.py's
mirror).  A variant's round is its resident batch on `cus` CUs (trio 40, pair 64, one-lane 256 txs per
CU at occupancy 1, 512 at occupancy 2); every size gives one sample (time / rounds, a partial round
counted whole), averaged.
  fit_auto.py SWEEP_JSON [CUS]"""
import json
import sys

PER = {"trio": 40, "pair": 64, "occ1": 256, "occ2": 512}


def fit(d, cus=256):
    out = {}
    for suite in ("secp", "sm2"):
        per_round = {}
        for v, per in PER.items():
            samples = []
            for k, ms in d.items():
                s, n, name = k.split("_")
                if s != suite or name != v:
                    continue
                n = int(n)
                rounds = -(-n // (per * cus))  # a partial round costs a whole one
                if v == "occ2" and n % (per * cus) and n % (per * cus) <= PER["occ1"] * cus:
                    continue  # (its short tail runs at occupancy-1 cost: not an occupancy-2 round)
                samples.append(ms / rounds)
            if samples:
                per_round[v] = sum(samples) / len(samples)
        if "trio" in per_round:
            t = per_round["trio"]
            out[suite] = {"ms_per_round": {k: round(v, 4) for k, v in per_round.items()},
                          "lat": {k: round(v / t, 3) for k, v in per_round.items()}}
    return out


if __name__ == "__main__":
    with open(sys.argv[1]) as f:
        line = [l for l in f.read().splitlines() if l.startswith("{")][-1]
    print(json.dumps(fit(json.loads(line), int(sys.argv[2]) if len(sys.argv) > 2 else 256), indent=1))
