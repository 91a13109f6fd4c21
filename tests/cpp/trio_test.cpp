// trio_test.cpp -- host build of ec26_trio.h / ecp26_trio.h with FE26_CHECK: the 16 lanes of one DPP row run as
// threads in lockstep (every DPP fetch / wave vote is a barrier), so the lane-trio doubling and mixed
// addition execute exactly as a wave does -- phantom lane 15 and the out-of-row zeros included -- while
// every field operation asserts its magnitude contract on every lane.  Each trio's result is compared
// with CurveK1x (ec26.h) -- or, for SM2, CurveSM2x (ecp26.h) -- on the same inputs: random elements at every magnitude the formulas accept,
// bound-hugging limbs, and the exceptional additions (P = Q, P = -Q, P = infinity, infinity doubled).
// Prints "trio ok <cases>" and exits 0, or the first mismatch and exits 1.
#define FE26_CHECK 1
#include "../../fisco-bcos_amd/csrc/ecp26_trio.h"

#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

using namespace bcosgpu;

namespace {
constexpr int kLanes = 16;
std::mutex mu;
std::condition_variable cv;
int arrived = 0;
unsigned long generation = 0;
uint32_t slot[kLanes];
thread_local int my_lane = 0;

void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const unsigned long g = generation;
    if (++arrived == kLanes) {
        arrived = 0;
        ++generation;
        cv.notify_all();
    } else {
        cv.wait(lk, [&] { return generation != g; });
    }
}
}  // namespace

namespace bcosgpu {
uint32_t trio_emu_dpp(uint32_t x, int ctrl) {
    slot[my_lane] = x;
    barrier();
    int src = my_lane;
    switch (ctrl) {
        case 0x111: src = my_lane - 1; break;  // row_shr:1
        case 0x112: src = my_lane - 2; break;  // row_shr:2
        case 0x101: src = my_lane + 1; break;  // row_shl:1
        case 0x102: src = my_lane + 2; break;  // row_shl:2
        default: abort();
    }
    const uint32_t r = (src >= 0 && src < kLanes) ? slot[src] : 0u;
    barrier();
    return r;
}
bool trio_emu_any(bool b) {
    slot[my_lane] = b ? 1u : 0u;
    barrier();
    bool r = false;
    for (int i = 0; i < kLanes; ++i) r = r || slot[i] != 0u;
    barrier();
    return r;
}
}  // namespace bcosgpu

namespace {
uint64_t rng_state = 0x2545f4914f6cdd1dull;
uint32_t rnd() {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return static_cast<uint32_t>(rng_state >> 11);
}
void rand_fe(fe26& a, int m, int mode) {  // mode 0 random limbs, 1 every limb at its bound
    for (int i = 0; i < 10; ++i) {
        const uint64_t bound = static_cast<uint64_t>(m) << (i == 9 ? 22 : 26);
        a.v[i] = static_cast<uint32_t>(mode ? bound : ((static_cast<uint64_t>(rnd()) << 20 ^ rnd()) % (bound + 1)));
    }
    a.m = m;
}
bool same(const fe26& a, const fe26& b) {
    fe26 x = a, y = b;
    fe26_normalize(x);
    fe26_normalize(y);
    return memcmp(x.v, y.v, sizeof x.v) == 0;
}
// the affine-equivalence of two Jacobian points (X1 Z2^2 = X2 Z1^2, Y1 Z2^3 = Y2 Z1^3) or both infinity
bool same_point(const Jac26& a, const Jac26& b) {
    if (a.inf || b.inf) return a.inf == b.inf;
    fe26 za2, zb2, za3, zb3, l, r;
    fe26_sqr(za2, a.Z);
    fe26_sqr(zb2, b.Z);
    fe26_mul(l, a.X, zb2);
    fe26_mul(r, b.X, za2);
    if (!same(l, r)) return false;
    fe26_mul(za3, za2, a.Z);
    fe26_mul(zb3, zb2, b.Z);
    fe26_mul(l, a.Y, zb3);
    fe26_mul(r, b.Y, za3);
    return same(l, r);
}

struct Case {
    Jac26 P;
    Aff26 Q;
    int ops;  // bit 0: 4 doublings, bit 1: one madd; repeated `reps` times
    int reps;
};
std::vector<Case> cases;
std::vector<int> bad;  // per case: 0 ok, 1 mismatch
int cases_per_round = 5;

void lane_main(int lane, int round) {
    my_lane = lane;
    const TrioLane T(lane);
    const int t = (lane % 16) / 3;
    const int c = round * cases_per_round + (t < 5 ? t : 4);
    const Case& K = cases[c];
    TrioPt P;
    trio::sel(P.S1, T.r0, K.P.X, K.P.Y);
    P.Xs = K.P.X;
    P.Zs = K.P.Z;
    P.inf = K.P.inf;
    Jac26 R = K.P;
    for (int rep = 0; rep < K.reps; ++rep) {
        if (K.ops & 1) {
            for (int d = 0; d < 4; ++d) {
                trio_dbl(P, T);
                CurveK1x::dbl(R, R);
            }
        }
        if (K.ops & 2) {
            trio_madd(P, P, K.Q, T);
            Jac26 S;
            CurveK1x::madd(S, R, K.Q);
            R = S;
        }
    }
    Jac26 J;
    trio_to_jac(J, P, T);
    if (t < 5 && !same_point(J, R)) bad[c] = 1;
}
// the GLV chain's window as the kernel runs it: 3 trio_dbl + trio_dbl_zz + trio_madd_zz (no P = +-Q
// tests, so no such cases), against 4 CurveK1x::dbl + CurveK1x::madd
std::vector<int> zbad;
void lane_main_zz(int lane, int round) {
    my_lane = lane;
    const TrioLane T(lane);
    const int t = (lane % 16) / 3;
    const int c = round * cases_per_round + (t < 5 ? t : 4);
    const Case& K = cases[c];
    TrioPt P;
    trio::sel(P.S1, T.r0, K.P.X, K.P.Y);
    P.Xs = K.P.X;
    P.Zs = K.P.Z;
    P.inf = K.P.inf;
    Jac26 R = K.P;
    for (int rep = 0; rep < K.reps; ++rep) {
        fe26 ZZ;
        trio_dbl(P, T);
        trio_dbl(P, T);
        trio_dbl(P, T);
        trio_dbl_zz(P, ZZ, T);
        trio_madd_zz(P, P, ZZ, K.Q, T);
        for (int d = 0; d < 4; ++d) CurveK1x::dbl(R, R);
        Jac26 S;
        CurveK1x::madd(S, R, K.Q);
        R = S;
    }
    Jac26 J;
    trio_to_jac(J, P, T);
    if (t < 5 && !same_point(J, R)) zbad[c] = 1;
}
// trio_add (Jacobian + Jacobian) against CurveK1x::add, chained `reps` times (R <- R + Q) so the
// outputs' magnitudes feed back in
struct CaseA {
    Jac26 P, Q;
    int reps;
};
std::vector<CaseA> acases;
std::vector<int> abad;

void to_trio(TrioPt& P, const Jac26& J, const TrioLane& T) {
    trio::sel(P.S1, T.r0, J.X, J.Y);
    P.Xs = J.X;
    P.Zs = J.Z;
    P.inf = J.inf;
}

void lane_main_add(int lane, int round) {
    my_lane = lane;
    const TrioLane T(lane);
    const int t = (lane % 16) / 3;
    const int c = round * cases_per_round + (t < 5 ? t : 4);
    const CaseA& K = acases[c];
    TrioPt P, Q;
    to_trio(P, K.P, T);
    to_trio(Q, K.Q, T);
    Jac26 R = K.P;
    for (int rep = 0; rep < K.reps; ++rep) {
        trio_add(P, P, Q, T);
        Jac26 S;
        CurveK1x::add(S, R, K.Q);
        R = S;
    }
    Jac26 J;
    trio_to_jac(J, P, T);
    if (t < 5 && !same_point(J, R)) abad[c] = 1;
}

// SM2: the same harness over fp26 / CurveSM2x (inputs X, Y <= 2, Z <= 8: what both ops accept)
void rand_fp(fp26& a, int m, int mode) {
    for (int i = 0; i < 10; ++i) {
        const uint64_t bound = static_cast<uint64_t>(m) << (i == 9 ? 22 : 26);
        a.v[i] = static_cast<uint32_t>(mode ? bound : ((static_cast<uint64_t>(rnd()) << 20 ^ rnd()) % (bound + 1)));
    }
    a.m = m;
}
bool same_p(const fp26& a, const fp26& b) {
    fp26 x = a, y = b;
    fp26_normalize(x);
    fp26_normalize(y);
    return memcmp(x.v, y.v, sizeof x.v) == 0;
}
bool same_point_p(const JacP26& a, const JacP26& b) {
    if (a.inf || b.inf) return a.inf == b.inf;
    fp26 za2, zb2, za3, zb3, l, r;
    fp26_sqr(za2, a.Z);
    fp26_sqr(zb2, b.Z);
    fp26_mul(l, a.X, zb2);
    fp26_mul(r, b.X, za2);
    if (!same_p(l, r)) return false;
    fp26_mul(za3, za2, a.Z);
    fp26_mul(zb3, zb2, b.Z);
    fp26_mul(l, a.Y, zb3);
    fp26_mul(r, b.Y, za3);
    return same_p(l, r);
}
struct CaseP {
    JacP26 P;
    AffP26 Q;
    int ops, reps;
};
std::vector<CaseP> pcases;
std::vector<int> pbad;

void lane_main_sm2(int lane, int round) {
    my_lane = lane;
    const TrioLane T(lane);
    const int t = (lane % 16) / 3;
    const int c = round * cases_per_round + (t < 5 ? t : 4);
    const CaseP& K = pcases[c];
    TrioPtP P;
    trio::sel(P.P1, T.r0, K.P.Z, K.P.Y);
    trio::sel(P.Q1, T.r1, K.P.Y, K.P.Z);
    P.Xr = K.P.X;
    P.inf = K.P.inf;
    JacP26 R = K.P;
    for (int rep = 0; rep < K.reps; ++rep) {
        if (K.ops & 1) {
            for (int d = 0; d < 4; ++d) {
                trio_dbl_sm2(P, T);
                CurveSM2x::dbl(R, R);
            }
        }
        if (K.ops & 2) {
            trio_madd_sm2(P, P, K.Q, T);
            JacP26 S;
            CurveSM2x::madd(S, R, K.Q);
            R = S;
        }
    }
    JacP26 J;
    trio_to_jac_sm2(J, P, T);
    if (t < 5 && !same_point_p(J, R)) pbad[c] = 1;
}
// the delta-carrying SM2 window: 4 trio_dbl_sm2_d + trio_madd_sm2_d (D = Z^2 travels with the point)
std::vector<int> pdbad;
void lane_main_sm2_d(int lane, int round) {
    my_lane = lane;
    const TrioLane T(lane);
    const int t = (lane % 16) / 3;
    const int c = round * cases_per_round + (t < 5 ? t : 4);
    const CaseP& K = pcases[c];
    TrioPtP P;
    trio::sel(P.P1, T.r0, K.P.Z, K.P.Y);
    trio::sel(P.Q1, T.r1, K.P.Y, K.P.Z);
    P.Xr = K.P.X;
    P.inf = K.P.inf;
    fp26 D;
    fp26_sqr(D, K.P.Z);
    JacP26 R = K.P;
    for (int rep = 0; rep < K.reps; ++rep) {
        for (int d = 0; d < 4; ++d) {
            trio_dbl_sm2_d(P, D, T);
            CurveSM2x::dbl(R, R);
        }
        fp26 Dn;
        trio_madd_sm2_d(P, Dn, P, D, K.Q, T);
        D = Dn;
        JacP26 S;
        CurveSM2x::madd(S, R, K.Q);
        R = S;
    }
    JacP26 J;
    trio_to_jac_sm2(J, P, T);
    bool ok = t >= 5 || same_point_p(J, R);
    if (t < 5 && ok && !R.inf) {  // D on lane 0 = Z^2 of the result (Z on lane 2 -> every lane of J)
        fp26 z2;
        fp26_sqr(z2, J.Z);
        ok = (T.r0 ? same_p(D, z2) : true);
    }
    if (t < 5 && !ok) pdbad[c] = 1;
}

// the window with a Jacobian table entry (trio_add_sm2_jd) against CurveSM2x::dbl / add, and D = Z^2
std::vector<JacEntP26> pqj;
std::vector<int> pjbad;
void lane_main_sm2_jd(int lane, int round) {
    my_lane = lane;
    const TrioLane T(lane);
    const int t = (lane % 16) / 3;
    const int c = round * cases_per_round + (t < 5 ? t : 4);
    const CaseP& K = pcases[c];
    const JacEntP26& Q = pqj[c];
    JacP26 QJ;
    QJ.X = Q.X;
    QJ.Y = Q.Y;
    QJ.Z = Q.Z;
    QJ.inf = false;
    TrioPtP P;
    trio::sel(P.P1, T.r0, K.P.Z, K.P.Y);
    trio::sel(P.Q1, T.r1, K.P.Y, K.P.Z);
    P.Xr = K.P.X;
    P.inf = K.P.inf;
    fp26 D;
    fp26_sqr(D, K.P.Z);
    JacP26 R = K.P;
    for (int rep = 0; rep < K.reps; ++rep) {
        for (int d = 0; d < 4; ++d) {
            trio_dbl_sm2_d(P, D, T);
            CurveSM2x::dbl(R, R);
        }
        fp26 Dn;
        trio_add_sm2_jd(P, Dn, P, D, Q, T);
        D = Dn;
        JacP26 S;
        CurveSM2x::add(S, R, QJ);
        R = S;
    }
    JacP26 J;
    trio_to_jac_sm2(J, P, T);
    bool ok = t >= 5 || same_point_p(J, R);
    if (t < 5 && ok && !R.inf) {
        fp26 z2;
        fp26_sqr(z2, J.Z);
        ok = (T.r0 ? same_p(D, z2) : true);
    }
    if (t < 5 && !ok) pjbad[c] = 1;
}
}  // namespace

int main() {
    // cases: random inputs at the largest magnitudes each entry accepts, bound-hugging limbs, and the
    // exceptional madd inputs (P = Q, P = -Q, P = inf; on rounds whose sequence starts with a madd) and
    // doubled infinities
    for (int k = 0; k < 400; ++k) {
        Case K;
        const int mode = k % 7 == 6 ? 1 : 0;
        const int mx = k % 3 == 0 ? 10 : 1 + static_cast<int>(rnd() % 10);
        rand_fe(K.P.X, mx, mode);
        rand_fe(K.P.Y, k % 3 == 0 ? 10 : 1 + static_cast<int>(rnd() % 10), mode);
        rand_fe(K.P.Z, k % 3 == 0 ? 16 : 1 + static_cast<int>(rnd() % 16), mode);
        rand_fe(K.Q.x, 1 + static_cast<int>(rnd() % 2), mode);
        rand_fe(K.Q.y, 1 + static_cast<int>(rnd() % 2), mode);
        K.P.inf = false;
        // the op sequence is uniform across the five trios of a row (one program counter per wave)
        const int round = k / cases_per_round;
        K.ops = 1 + round % 3;
        K.reps = 1 + round % 4;
        const int special = k % 10;
        if (special == 1 || special == 2) {  // P = (x Z^2, +-y Z^3, Z) equals +-Q
            fe26 z2, z3;
            rand_fe(K.P.Z, 2, 0);
            rand_fe(K.Q.x, 1, 0);
            rand_fe(K.Q.y, 1, 0);
            fe26_sqr(z2, K.P.Z);
            fe26_mul(z3, z2, K.P.Z);
            fe26_mul(K.P.X, K.Q.x, z2);
            fe26_mul(K.P.Y, K.Q.y, z3);
            if (special == 2) fe26_neg<2>(K.P.Y, K.P.Y);
        } else if (special == 3) {  // P = infinity
            CurveK1x::set_inf(K.P);
        }
        cases.push_back(K);
    }
    bad.assign(cases.size(), 0);
    const int rounds = static_cast<int>(cases.size()) / cases_per_round;
    for (int r = 0; r < rounds; ++r) {
        std::vector<std::thread> th;
        for (int l = 0; l < kLanes; ++l) th.emplace_back(lane_main, l, r);
        for (auto& x : th) x.join();
    }
    // the zz window over the same inputs, minus the P = +-Q cases (kept as plain random inputs)
    {
        std::vector<Case> saved = cases;
        for (size_t k = 0; k < cases.size(); ++k)
            if (k % 10 == 1 || k % 10 == 2) rand_fe(cases[k].P.Z, 3, 0);  // P no longer +-Q
        zbad.assign(cases.size(), 0);
        for (int r = 0; r < rounds; ++r) {
            std::vector<std::thread> th;
            for (int l = 0; l < kLanes; ++l) th.emplace_back(lane_main_zz, l, r);
            for (auto& x : th) x.join();
        }
        int nz = 0;
        for (size_t i = 0; i < zbad.size(); ++i)
            if (zbad[i]) {
                if (!nz) printf("zz window mismatch in case %zu (reps %d)\n", i, cases[i].reps);
                ++nz;
            }
        if (nz) {
            printf("trio zz mismatches %d of %zu\n", nz, cases.size());
            return 1;
        }
        cases = saved;
    }
    for (int k = 0; k < 300; ++k) {
        CaseA K;
        const int mode = k % 7 == 6 ? 1 : 0;
        rand_fe(K.P.X, k % 3 == 0 ? 16 : 1 + static_cast<int>(rnd() % 16), mode);
        rand_fe(K.P.Y, k % 3 == 0 ? 16 : 1 + static_cast<int>(rnd() % 16), mode);
        rand_fe(K.P.Z, k % 3 == 0 ? 16 : 1 + static_cast<int>(rnd() % 16), mode);
        rand_fe(K.Q.X, k % 3 == 0 ? 16 : 1 + static_cast<int>(rnd() % 16), mode);
        rand_fe(K.Q.Y, k % 3 == 0 ? 16 : 1 + static_cast<int>(rnd() % 16), mode);
        rand_fe(K.Q.Z, k % 3 == 0 ? 16 : 1 + static_cast<int>(rnd() % 16), mode);
        K.P.inf = K.Q.inf = false;
        K.reps = 1 + (k / cases_per_round) % 3;
        const int special = k % 10;
        if (special == 1 || special == 2) {  // Q = (X l^2, +-Y l^3, Z l): the same point as +-P
            fe26 l, l2, l3;
            rand_fe(l, 1, 0);
            rand_fe(K.P.X, 2, 0);
            rand_fe(K.P.Y, 2, 0);
            rand_fe(K.P.Z, 2, 0);
            fe26_sqr(l2, l);
            fe26_mul(l3, l2, l);
            fe26_mul(K.Q.X, K.P.X, l2);
            fe26_mul(K.Q.Y, K.P.Y, l3);
            fe26_mul(K.Q.Z, K.P.Z, l);
            if (special == 2) fe26_neg<2>(K.Q.Y, K.Q.Y);
        } else if (special == 3) {
            CurveK1x::set_inf(K.P);
        } else if (special == 4) {
            CurveK1x::set_inf(K.Q);
        } else if (special == 5) {
            CurveK1x::set_inf(K.P);
            CurveK1x::set_inf(K.Q);
        }
        acases.push_back(K);
    }
    abad.assign(acases.size(), 0);
    for (int r = 0; r < static_cast<int>(acases.size()) / cases_per_round; ++r) {
        std::vector<std::thread> th;
        for (int l = 0; l < kLanes; ++l) th.emplace_back(lane_main_add, l, r);
        for (auto& x : th) x.join();
    }
    int nabad = 0;
    for (size_t i = 0; i < abad.size(); ++i)
        if (abad[i]) {
            if (!nabad) printf("add mismatch in case %zu (reps %d)\n", i, acases[i].reps);
            ++nabad;
        }
    if (nabad) {
        printf("trio add mismatches %d of %zu\n", nabad, acases.size());
        return 1;
    }
    for (int k = 0; k < 300; ++k) {
        CaseP K;
        const int mode = k % 7 == 6 ? 1 : 0;
        rand_fp(K.P.X, k % 3 == 0 ? 2 : 1 + static_cast<int>(rnd() % 2), mode);
        rand_fp(K.P.Y, k % 3 == 0 ? 2 : 1 + static_cast<int>(rnd() % 2), mode);
        rand_fp(K.P.Z, k % 3 == 0 ? 8 : 1 + static_cast<int>(rnd() % 8), mode);
        rand_fp(K.Q.x, 1 + static_cast<int>(rnd() % 2), mode);
        rand_fp(K.Q.y, 1 + static_cast<int>(rnd() % 2), mode);
        K.P.inf = false;
        const int round = k / cases_per_round;
        K.ops = 1 + round % 3;
        K.reps = 1 + round % 4;
        const int special = k % 10;
        if (special == 1 || special == 2) {  // P = (x Z^2, +-y Z^3, Z) equals +-Q
            fp26 z2, z3;
            rand_fp(K.P.Z, 2, 0);
            rand_fp(K.Q.x, 1, 0);
            rand_fp(K.Q.y, 1, 0);
            fp26_sqr(z2, K.P.Z);
            fp26_mul(z3, z2, K.P.Z);
            fp26_mul(K.P.X, K.Q.x, z2);
            fp26_mul(K.P.Y, K.Q.y, z3);
            if (special == 2) {
                fp26_neg<2>(K.P.Y, K.P.Y);
                fp26_normalize_weak(K.P.Y);
            }
        } else if (special == 3) {
            CurveSM2x::set_inf(K.P);
        }
        pcases.push_back(K);
    }
    pbad.assign(pcases.size(), 0);
    for (int r = 0; r < static_cast<int>(pcases.size()) / cases_per_round; ++r) {
        std::vector<std::thread> th;
        for (int l = 0; l < kLanes; ++l) th.emplace_back(lane_main_sm2, l, r);
        for (auto& x : th) x.join();
    }
    {  // the delta-carrying window over the same inputs, minus the P = +-Q cases
        std::vector<CaseP> saved = pcases;
        for (size_t k = 0; k < pcases.size(); ++k)
            if (k % 10 == 1 || k % 10 == 2) rand_fp(pcases[k].P.Z, 3, 0);
        pdbad.assign(pcases.size(), 0);
        for (int r = 0; r < static_cast<int>(pcases.size()) / cases_per_round; ++r) {
            std::vector<std::thread> th;
            for (int l = 0; l < kLanes; ++l) th.emplace_back(lane_main_sm2_d, l, r);
            for (auto& x : th) x.join();
        }
        int nd = 0;
        for (size_t i = 0; i < pdbad.size(); ++i)
            if (pdbad[i]) {
                if (!nd) printf("sm2 delta window mismatch in case %zu (reps %d)\n", i, pcases[i].reps);
                ++nd;
            }
        if (nd) {
            printf("trio sm2 delta mismatches %d of %zu\n", nd, pcases.size());
            return 1;
        }
        // the Jacobian-entry window over the same inputs (Q: random X, Y, Z with its Z powers)
        pqj.clear();
        for (size_t k = 0; k < pcases.size(); ++k) {
            JacEntP26 E;
            rand_fp(E.X, 1, k % 7 == 6 ? 1 : 0);
            rand_fp(E.Y, 1, 0);
            rand_fp(E.Z, 1, 0);
            fp26_sqr(E.ZZ, E.Z);
            fp26_mul(E.ZZZ, E.ZZ, E.Z);
            pqj.push_back(E);
        }
        pjbad.assign(pcases.size(), 0);
        for (int r = 0; r < static_cast<int>(pcases.size()) / cases_per_round; ++r) {
            std::vector<std::thread> th;
            for (int l = 0; l < kLanes; ++l) th.emplace_back(lane_main_sm2_jd, l, r);
            for (auto& x : th) x.join();
        }
        int nj = 0;
        for (size_t i = 0; i < pjbad.size(); ++i)
            if (pjbad[i]) {
                if (!nj) printf("sm2 jacobian-entry window mismatch in case %zu (reps %d)\n", i, pcases[i].reps);
                ++nj;
            }
        if (nj) {
            printf("trio sm2 jacobian-entry mismatches %d of %zu\n", nj, pcases.size());
            return 1;
        }
        pcases = saved;
    }
    int npbad = 0;
    for (size_t i = 0; i < pbad.size(); ++i)
        if (pbad[i]) {
            if (!npbad) printf("sm2 mismatch in case %zu (ops %d reps %d)\n", i, pcases[i].ops, pcases[i].reps);
            ++npbad;
        }
    if (npbad) {
        printf("trio sm2 mismatches %d of %zu\n", npbad, pcases.size());
        return 1;
    }
    int nbad = 0;
    for (size_t i = 0; i < bad.size(); ++i)
        if (bad[i]) {
            if (!nbad) printf("mismatch in case %zu (ops %d reps %d)\n", i, cases[i].ops, cases[i].reps);
            ++nbad;
        }
    if (nbad) {
        printf("trio mismatches %d of %zu\n", nbad, cases.size());
        return 1;
    }
    printf("trio ok %zu secp256k1 + %zu zz windows + %zu secp256k1 add + %zu sm2 + %zu sm2 delta windows + %zu sm2 "
           "jacobian-entry windows\n",
           cases.size(), cases.size(), acases.size(), pcases.size(), pcases.size(), pcases.size());
    return 0;
}
