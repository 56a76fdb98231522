// mh_chain.hip -- MI355X (gfx950) Metropolis-Hastings interior-layout chains.
//
// Rebuilds the reference's per-chain hot path (KernelFolder/Kernel/Kernel.cu:754-871: propose
// :576-704, Costs :516-550, Accept :706-713) for CDNA4:
//   * a chain is a group of L lanes (L = 64 -> one wavefront per chain; L = 8..32 for small
//     rooms, 64/L chains per wavefront); each lane owns objects r, r+L, r+2L, ...;
//   * the chain's configuration lives in LDS for the whole launch; the proposal edits at most
//     two objects IN PLACE and a rejected proposal is undone from a register backup (the
//     reference copies the whole configuration twice per step, Kernel.cu:792,824);
//   * the O(N^2) symmetry rows and the O(C*N) clearance pairs are spread over the lanes; the
//     reference's float/double sums are replayed serially in the reference's order through
//     readlane/ds_bpermute (so results are bit-identical, not merely close), skipping exact
//     zeros (x - 0 == x);
//   * OffLimitsCosts never enters totalCosts (Kernel.cu:547) and so cannot change a decision:
//     it is evaluated once, for the final state only;
//   * the RNG is rocRAND's Philox4x32-10 (seed, subsequence = global chain id), resumable by
//     draw count, so k launches of m steps equal one launch of k*m steps.
// Compiled with -ffp-contract=off: every multiply and add rounds where the reference's does.

#include <stdint.h>
#include <stdlib.h>

#include "mh_common.h"
#ifndef MH_CHAIN_STEP_TU
#include <rocrand/rocrand_xorwow.h>
#endif
#ifndef MH_DOUBLE
#define MH_DOUBLE 0  // cost-probe builds: run phase k twice when bit k is set; product = 0
                     // (1 A, 2 full symmetry, 64 delta symmetry, 4 SA, 8 CL, 16 PW/ANG, 32 replay,
                     // 128 Clearance pair update, 256 the rejection bound's lane terms and sums)
#endif
#define MH_REPS(bit) ((MH_DOUBLE & (bit)) ? 2 : 1)
#define MH_CLOBBER() asm volatile("" ::: "memory")
#ifndef MH_STAMPS
#define MH_STAMPS 0  // diagnostic builds (tools/build_stamps.sh) time each phase; product = 0
#endif

#if MH_STAMPS
#ifdef MH_CHAIN_STEP_TU
static __device__ unsigned long long g_phase_cycles[16];  // (XORWOW kernels: not reported)
#else
__device__ unsigned long long g_phase_cycles[16];
#endif
#define MH_STAMP(t) do { __builtin_amdgcn_sched_barrier(0); asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory"); __builtin_amdgcn_sched_barrier(0); } while (0)
#define MH_PHASE(ch, k, t0) do { unsigned long long _t; MH_STAMP(_t); stage((ch).aux)->cyc[k] += _t - (t0); (t0) = _t; } while (0)
#else
#define MH_STAMP(t) do { } while (0)
#define MH_PHASE(ch, k, t0) do { } while (0)
#endif

namespace mh {

struct Backup {  // the cost-relevant pose of one object (z, rotX, rotZ never enter a cost)
    int k;
    double x, y, ry;
};

// Per-chain scalars kept in LDS rather than registers while the costs are evaluated.
struct ChainAux {
    Backup b[2];
    int nb;       // backups in use (0, 1 or 2)
    int swap_a, swap_b;  // a swap proposal's objects (-1: none); z/rotX/rotZ swap in HBM on accept
    float cur[8]; // resultCosts of the current configuration
    float star[8];  // resultCosts of the proposal, when exact (the step keeps only its total in a
                    // register: held across the rare exact current pass, the eight spilled)
    uint64_t rng_key[3];  // the Philox stream's seed and subsequence, the window's first draw
                          // (WaveRngLds::ss)
#if MH_STAMPS
    unsigned long long cyc[12];  // diagnostic: cycles per phase (writer lane); [8] steps that
                                 // evaluated the bound, [9] steps it rejected, [10] steps it
                                 // accepted, [11] exact evaluations of the current configuration
#endif
};
static_assert(sizeof(ChainAux) <= kChainAuxBytes, "ChainAux");

// The double pose (x, y, rotY) of the objects this lane owns, m * L + r for m < NPL, kept in
// registers for the whole launch: every cost term reads a lane's own objects, and the few
// reads of another object's pose (the proposal's objects, a symmetry row's leader column) go
// lane to lane. LDS keeps only the float pose words (ObjP) that the O(N^2) scans read.
template <int NPL>
struct OwnPose {
    double x[NPL], y[NPL], ry[NPL];
};

// rotY of object j, group-uniform j: from its owner lane (readlane / ds_bpermute).
template <int L, int NPL>
__device__ __forceinline__ double pose_ry(const OwnPose<NPL>& op, int j, int gbase) {
    return grp_get<L>(sel<NPL>(op.ry, j / L), j % L, gbase);
}

// rotY of object j where j differs between lanes (j < 0 reads object 0): one ds_bpermute per
// owned slot, then the slot's value. Call with every lane of the wavefront active.
template <int L, int NPL>
__device__ __forceinline__ double pose_ry_var(const OwnPose<NPL>& op, int j, int gbase) {
    const int jj = j < 0 ? 0 : j;
    const int addr = (gbase + jj % L) << 2;
    const int slot = jj / L;
    double out = 0.0;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
        const double o = __hiloint2double(__builtin_amdgcn_ds_bpermute(addr, __double2hiint(op.ry[m])),
                                          __builtin_amdgcn_ds_bpermute(addr, __double2loint(op.ry[m])));
        out = (m == slot) ? o : out;
    }
    return out;
}

// The chain's LDS. Every array that one lane writes and other lanes read is a Published view
// (mh_common.h): lanes write through stage(ch.X), and each phase ends in hand_off(ch.X, ...).
struct ChainPtrs {
    const RectShape* objs;  // room tables, staged once per workgroup into LDS (ChainLds)
    const RectShape* clrs;
    const RelConst* relc;
    const uint2* rix;  // [R] relationship i's objects {s | t << 16, as | at << 16}
    const float4* re0;  // [R] fp32 constants of the relationships' estimates (rel_est_consts)
    const float4* re1;
    Published<ObjP> P;
    Published<double> PX, PY;  // [N4] per-object double terms of the dense ordered sums (zero past N)
    Published<double> CPHF, RMXF;  // [N4] per-object float terms (-cos phi, -row max), widened
    Published<double> LCL;  // compacted non-zero Clearance terms (float values), capacity 2L
    Published<double> LPW;  // compacted non-zero PairWise / Angle terms, capacity lst_r each
    Published<double> LANG;
    int lst_r;
    double* zrr;      // HBM: this chain's z, rotX, rotZ rows (F_Z, F_RX, F_RZ of the pose block)
    Published<float4> OFF;
    Published<float4> CLA;
    Published<uint64_t> NZ;  // [2][C] row words of the non-zero Clearance pairs
    Published<int> PRE;      // [C] row prefix counts
    Published<ChainAux> aux;  // (the writer lane's record)
    const DevRoom* rm;  // LDS copy of the room scalars
    const double* zero4;  // four zero doubles (a finished replay lane reads these)
};

// ---- compacted term lists for the ordered sums -------------------------------------------
//
// Clearance terms (floats, capacity 2L) and PairWise / Angle terms (doubles, capacity lst_r =
// min(L, R) each) are compacted in the reference's order into LDS lists. Lane 4 (Clearance),
// 6 (PairWise) and 7 (Angle) of the group own those sums; a list that would overflow is first
// folded into its owner's accumulator (only for pathologically overlapping rooms).

template <typename T>
__device__ __forceinline__ void list_flush(const Staged<T>& buf, int& cnt, double& acc, bool owner,
                                           bool to_float) {
    const Published<T> v = publish(buf);  // (every lane's appends)
    if (owner) {
        for (int l = 0; l < cnt; ++l) {
            const double t = acc + (double)v[l];
            acc = to_float ? (double)(float)t : t;
        }
    }
    cnt = 0;
    (void)restage(v);  // (the owner's reads are done before any lane appends again)
}

// Appends, in lane order, the value of every lane whose `nz` is set (folding the list into its
// owner's accumulator first only if these values would not fit).
template <int L, typename T>
__device__ __forceinline__ void list_append(const Staged<T>& buf, int cap, int& cnt, double& acc,
                                            bool owner, bool to_float, T v, bool nz, int r,
                                            int gbase) {
    const uint64_t b = group_ballot<L>(nz, gbase);
    const int add = __builtin_popcountll(b);
    if (add == 0) return;
    if (cnt + add > cap) list_flush(buf, cnt, acc, owner, to_float);
    if (nz) buf.put(cnt + __builtin_popcountll(b & ((1ull << r) - 1ull)), v);
    cnt += add;
}

// Appends K values per lane in order k = 0..K-1 (each in lane order): one overflow test and
// one count update for the batch.
template <int L, int K, typename T>
__device__ __forceinline__ void list_append_n(const Staged<T>& buf, int cap, int& cnt, double& acc,
                                              bool owner, bool to_float, const T (&v)[K],
                                              const bool (&nz)[K], int r, int gbase) {
    uint64_t b[K];
    int add = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        b[k] = group_ballot<L>(nz[k], gbase);
        add += __builtin_popcountll(b[k]);
    }
    if (add == 0) return;
    if (cnt + add > cap) list_flush(buf, cnt, acc, owner, to_float);
    const uint64_t below = (1ull << r) - 1ull;
    int pos = cnt;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (nz[k]) buf.put(pos + __builtin_popcountll(b[k] & below), v[k]);
        pos += __builtin_popcountll(b[k]);
    }
    cnt = pos;
}

// PairWiseCosts (:210-233) and PairWiseAngleCosts (:236-263) terms of relationship q (mh_common.h).
__device__ __forceinline__ void rel_terms(const ChainPtrs& ch, int q, double& tpw, double& tang) {
    rel_terms(ch.relc[q], ch.P.ptr(), tpw, tang);
}

// ---- FocalPoint and relationship terms of one lane, exact or estimated ------------------------
//
// Steps with one object per lane: lane i holds object i's FocalPoint term and relationship i's
// PairWise / PairWiseAngle terms. exact_terms() evaluates them as the reference does (double
// atan2, double cos rounded to float, double distance and divisions, Kernel.cu:170-188,
// 210-281); one shared atan2 pass serves a lane's relationship or, failing that, its object, and
// a lane that needs both takes a second (rare) pass.
__device__ __forceinline__ void exact_terms(const ChainPtrs& ch, const DevRoom& rm, int i, int n,
                                            bool obj, bool rel, float& cph, double& rpw,
                                            double& rang) {
    const ObjP p = ch.P[i < n ? i : 0];
    const double fy = (double)(rm.fyf - p.yf), fx = (double)(rm.fxf - p.xf);
    double dy = fy, dx = fx, tpw = 0.0;
    float ti = 0.0f;
    if (rel) tpw = rel_pair(ch.relc[i], ch.P.ptr(), dy, dx, ti);
    double a1 = 0.0, a2 = 0.0;
    if (rel || obj) a1 = atan2_ool(dy, dx);
    if (rel && obj) a2 = atan2_ool(fy, fx);
    if (obj) {
        const float at = (float)(rel ? a2 : a1);
        const float b = at - p.rotYf;
        const float ph = (float)((double)b + kHalfPI);
        cph = cos_f32(ph);
    }
    if (rel) {
        rpw = tpw;
        rang = rel_angle(ch.relc[i], a1, ti);
    }
}

// (rel_pw_est, rel_ang_est: mh_common.h, shared with the incremental kernel)

// fp32 estimates of the same terms for the rejection bound (no double arithmetic, no division,
// no library transcendental): cph within kDeltaCph, rpw within kPwEstU U relative, rang within
// eang (returned). `amb` (relationship) / `ambo` (object) are set where the estimate lies too
// near one of the reference's discontinuities for its branch to be certain -- the distance
// range's ends (:216-221), theta's two wraps (:176-181), the wrapped range's fmodf and switch
// (:245-250) -- or outside the ranges the allowances are derived for (mh_common.h kDeltaCph);
// such a lane needs exact_terms(). Relationship i's objects come from rix[i] (16-bit indices).
__device__ __forceinline__ void rel_objs(const ChainPtrs& ch, int i, ObjP& ps, ObjP& pt, ObjP& as,
                                         ObjP& atp) {
    const uint2 q = ch.rix[i];
    ps = ch.P[q.x & 0xffffu];
    pt = ch.P[q.x >> 16];
    as = ch.P[q.y & 0xffffu];
    atp = ch.P[q.y >> 16];
}

// (cph_est: mh_common.h)

template <bool SHARE>
__device__ __forceinline__ void approx_terms(const ChainPtrs& ch, const DevRoom& rm, int i, int n,
                                             bool obj, bool rel, float& cph, double& rpw,
                                             double& rang, float& eang, bool& amb, bool& ambo) {
    constexpr float TINY = 0x1p-100f;  // (atan2_est's domain)
    if constexpr (!SHARE) {
        // (the latency-bound few-chains instance: two passes, the object's first -- 4.20
        // against 4.24 ms per config-2 launch with the shared pass)
        if (obj) {
            const ObjP p = ch.P[i < n ? i : 0];
            const float fy = rm.fyf - p.yf, fx = rm.fxf - p.xf;
            ambo |= !(fmaxf(fabsf(fy), fabsf(fx)) >= TINY);
            cph = cph_est(atan2_est(fy, fx), p, ambo);
        }
        if (rel) {
            ObjP ps, pt, as, atp;
            rel_objs(ch, i, ps, pt, as, atp);
            const float4 e0 = ch.re0[i], e1 = ch.re1[i];
            rpw = rel_pw_est(e0, ps, pt, amb);
            const float ay = as.yf - atp.yf, ax = as.xf - atp.xf;
            amb |= !(fmaxf(fabsf(ay), fabsf(ax)) >= TINY);
            rang = rel_ang_est(e1, e0.w, atp, atan2_est(ay, ax), eang, amb);
        }
        return;
    }
    // One atan2 pass serves a relationship lane's angle (theta) or, failing that, an object
    // lane's focal angle; a lane needing both (its object moved and its relationship was touched)
    // takes a second pass (config 3: 115.2 -> 114.4 ms per launch).
    const ObjP p = ch.P[i < n ? i : 0];
    const float fy = rm.fyf - p.yf, fx = rm.fxf - p.xf;
    float ay = fy, ax = fx;
    float4 e0 = make_float4(0.f, 0.f, 0.f, 0.f), e1 = e0;
    ObjP atp;
    if (rel) {
        ObjP ps, pt, as;
        rel_objs(ch, i, ps, pt, as, atp);
        e0 = ch.re0[i];
        e1 = ch.re1[i];
        rpw = rel_pw_est(e0, ps, pt, amb);
        ay = as.yf - atp.yf;
        ax = as.xf - atp.xf;
    }
    const bool tiny = !(fmaxf(fabsf(ay), fabsf(ax)) >= TINY);
    const float a1 = atan2_est(ay, ax);
    float at = a1;
    if (obj && rel) {
        at = atan2_est(fy, fx);
        ambo |= !(fmaxf(fabsf(fy), fabsf(fx)) >= TINY);
    } else if (obj) {
        ambo |= tiny;
    }
    if (obj) cph = cph_est(at, p, ambo);
    if (rel) {
        amb |= tiny;
        rang = rel_ang_est(e1, e0.w, atp, a1, eang, amb);
    }
}

// ---- incremental Clearance pairs (one object per lane) ---------------------------------------
//
// A proposal changes the pairs of the moved objects' columns and of the rows of clearances they
// carry; the others keep their zero / non-zero state. Updates this lane's column mask and the
// proposed row words (the other LDS buffer), writes the row prefix counts of the proposed rows
// and returns the number of non-zero pairs (Kernel.cu:408-431 terms that are not exactly zero).
template <int L>
__device__ __forceinline__ int inc_cl_update(const ChainPtrs& ch, int n, int c, int ka, int kb,
                                             int r, int gbase, float4 boxj, const ClPairs& clp,
                                             ClPairs& clo, bool& colchg) {
    const int j = r;
    const uint64_t* NZc = ch.NZ.ptr() + clp.buf * c;
    const Staged<uint64_t> NZn = stage(ch.NZ.at((clp.buf ^ 1) * c));
    uint64_t cm = clp.cm;
    uint64_t w = (r < c) ? NZc[r] : 0ull;  // lane r's clearance row, patched below
    const int kk2[2] = {ka, kb};
#pragma unroll
    for (int q = 0; q < 2; ++q) {  // the moved objects' columns, one clearance per lane
        const int k = kk2[q];
        if (k < 0) continue;
        const ObjP pk = ch.P[k];
        const float4 bk = shape_box(ch.objs[k], pk.xf, pk.yf);
        const bool nzk = r < c && overlap(ch.CLA[r], bk) != 0.0f;
        const uint64_t colk = group_ballot<L>(nzk, gbase);
        if (j == k) cm = colk;
        w = (w & ~(1ull << k)) | ((uint64_t)nzk << k);
    }
    // rows of the clearances whose source moved: every object lane re-tests its pair
    uint64_t moved = group_ballot<L>(r < c && (ch.clrs[r].pad == ka || ch.clrs[r].pad == kb),
                                     gbase);
    while (moved) {
        const int i = __builtin_ctzll(moved);
        moved &= moved - 1;
        const bool nzi = j < n && overlap(ch.CLA[i], boxj) != 0.0f;
        const uint64_t row = group_ballot<L>(nzi, gbase);
        colchg = colchg || nzi || ((cm >> i) & 1ull) != 0;  // (the pair before or after)
        cm = (cm & ~(1ull << i)) | ((uint64_t)nzi << i);
        if (r == i) w = row;
    }
    if (r < c) NZn.put(r, w);
    int total;
    const int pre = group_excl_scan<L>(r < c ? __builtin_popcountll(w) : 0, r, total);
    if (r < c) stage(ch.PRE).put(r, pre);
    clo.cm = cm;
    clo.buf = clp.buf ^ 1;
    hand_off(ch.NZ, ch.PRE);  // the proposed rows and their prefix counts: the list build's
    return total;
}

// ---- Costs(), Kernel.cu:516-550, for the configuration currently in LDS --------------------
//
// Every lane of the group returns the same costs. out: resultCosts order
// {total, PW, VB, FP, SYM, CL, OL, SA}. `sym` returns the symmetry row maxima of the evaluated
// configuration. With DELTA, `prev` holds them for the configuration before the proposal, which
// differs from the evaluated one only in objects ka and kb (-1: none), and only the rows and
// columns those objects touch are re-evaluated.
// FAST (steps without best-of-chain tracking, one chain per wavefront): before any ordered sum
// is built, the proposal's total is bounded from lane-parallel sums (bound_decide, against the
// current total's interval `cur`) and, when the bound already decides Accept for the drawn
// uniform `u_acc`, the function returns with *fast set to BOUND_REJECT or BOUND_ACCEPT, the
// proposal's interval in *star_iv and `out` unset (the symmetry rows and Clearance pairs are
// set: they come before the bound); otherwise it goes on to the exact costs.
// eval_costs and propose are always inlined into the step kernels: an out-of-line call that
// takes references to the kernel's private (stack) objects faulted on MI355X with this toolchain
// (DESIGN.md "The counting-build fault"; round 2's MH_STAMPS build, where the inliner left
// eval_costs out of line). tests/test_abi.py checks that no kernel calls either.
// MH_EVAL_INLINE=-1 builds the out-of-line variant for that experiment.
#ifndef MH_EVAL_INLINE
#define MH_EVAL_INLINE 1
#endif
#if MH_EVAL_INLINE > 0
#define MH_EVAL_ATTR __attribute__((always_inline))
#else
#define MH_EVAL_ATTR __attribute__((noinline))
#endif

template <int L, int NPL, bool WITH_OL, bool DELTA, bool FAST = false, bool PAIRS = false>
__device__ MH_EVAL_ATTR void eval_costs(const LaunchArgs& a, const ChainPtrs& ch, const OwnPose<NPL>& op,
                           int r, int gbase,
                           float out[8], SymRows<NPL>& sym, const SymRows<NPL>& prev, int ka,
                           int kb, ClPairs& clo, const ClPairs& clp, float u_acc = 0.0f,
                           CostIv cur = CostIv{0.0f, 0.0f}, int* fast = nullptr,
                           CostIv* star_iv = nullptr, bool save = false) {
    // The room scalars are read from the workgroup's LDS copy where they are used, not kept
    // live in SGPRs from the kernel arguments (that spilled ~140 SGPRs into VGPR lanes).
    // (the few-chains instance reads them from the kernel arguments: no LDS round trip on its
    // latency-bound step; config 2 4.30 -> 4.25 ms per 1,000-step launch)
    const DevRoom& rm = PAIRS ? a.rm : *ch.rm;
    const int n = a.rm.n, c = a.rm.c;

    unsigned long long t0 = 0;
    MH_STAMP(t0);
    // Phase A: per-object and per-clearance terms of the owned slots. Steps with one object per
    // lane keep terms across steps and share one atan2 pass (below); the 8-lane instance (rooms
    // of up to 8 objects: latency-bound, few chains) keeps the direct per-lane passes.
    constexpr bool SHARED = DELTA && NPL == 1 && L >= 16;
    float px[NPL], py[NPL];  // the VisualBalance products rounded to float (the bound's terms)
    float cph[NPL], rxs[NPL], rys[NPL], rrs[NPL];
    float4 sao[NPL], sac[NPL];
    float4 boxo[NPL];  // each owned object's box at its pose (SurfaceArea, Clearance pairs)
    double rpw[NPL], rang[NPL];  // relationship terms of chunks m < NPL (see Phase F)
    bool wild = false;  // a pose outside the range the fp32 symmetry estimate is proven for
    for (int rep = 0; rep < MH_REPS(1); ++rep) {
    MH_CLOBBER();
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
        const int i = m * L + r;
        px[m] = py[m] = 0.0f;
        cph[m] = rxs[m] = rys[m] = rrs[m] = 0.0f;
        rpw[m] = rang[m] = 0.0;
        sao[m] = sac[m] = boxo[m] = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (SHARED) {
            // Steps, one object per lane: only the moved objects' FocalPoint terms and the
            // relationships they touch change; the rest keep their terms (clp). Steps that
            // decide on the rejection bound (FAST) take fp32 estimates of the changed terms and
            // mark them (dc, dr); exact passes evaluate every marked or changed term exactly.
            // (This runs first, so the per-object values below are not live across the atan2.)
            const bool moved = i < n && (i == ka || i == kb) && !(MH_ABLATE & 2);
            bool touched = false;
            if (i < rm.r && !(MH_ABLATE & 16)) {
                const uint2 q = ch.rix[i];
                const unsigned a16 = (unsigned)ka, b16 = (unsigned)kb;  // (ka, kb < 65536)
                touched = ka >= 0 && ((q.x & 0xffffu) == a16 || (q.x >> 16) == a16 ||
                                      (q.y & 0xffffu) == a16 || (q.y >> 16) == a16 ||
                                      (q.x & 0xffffu) == b16 || (q.x >> 16) == b16 ||
                                      (q.y & 0xffffu) == b16 || (q.y >> 16) == b16);
            }
            cph[m] = clp.cph;
            rpw[m] = clp.rpw;
            rang[m] = clp.rang;
            clo.dc = clp.dc;
            clo.dr = clp.dr;
            clo.eang = clp.eang;
            if constexpr (FAST) {
                bool amb = false, ambo = false;
                if (__ballot(moved || touched))
                    approx_terms<!PAIRS>(ch, rm, i, n, moved, touched, cph[m], rpw[m], rang[m], clo.eang,
                                 amb, ambo);
                clo.dc = clo.dc || moved;
                clo.dr = clo.dr || touched;
                if (__ballot(amb || ambo)) {  // (rare) an estimate near a discontinuity: exact
                    if (amb) {
                        clo.dr = false;
                        clo.eang = 0.0f;
                    }
                    if (ambo) clo.dc = false;
                    exact_terms(ch, rm, i, n, ambo, amb, cph[m], rpw[m], rang[m]);
                }
            } else {
                const bool obj = moved || (i < n && clp.dc);
                const bool rel = touched || (i < rm.r && clp.dr);
                if (__ballot(obj || rel)) exact_terms(ch, rm, i, n, obj, rel, cph[m], rpw[m], rang[m]);
                clo.dc = clo.dr = false;
                clo.eang = 0.0f;
            }
        }
        if (i < n) {
            const RectShape os = ch.objs[i];
            const float area = __int_as_float(os.pad);
            const ObjP p = ch.P[i];
            const double x = op.x[m], y = op.y[m];
            wild |= !(fabs(x) < 1e15 && fabs(y) < 1e15 && fabs(op.ry[m]) < 1e15);
            // VisualBalanceCosts products, Kernel.cu:200-201.
            // (to the replay's LDS streams at once: held in registers to the replay, the
            // doubles spilled on the exact paths)
            const double vx = (double)area * x, vy = (double)area * y;
            stage(ch.PX).put(i, vx);
            stage(ch.PY).put(i, vy);
            px[m] = (float)vx;
            py[m] = (float)vy;
            // FocalPointCosts term, Kernel.cu:271,277 with phi() of :185-188 (steps with one
            // object per lane: above, sharing the relationship terms' atan2 pass).
            if (!(MH_ABLATE & 2) && !SHARED) {
                float at = atan2_f32(rm.fyf - p.yf, rm.fxf - p.xf);
                float b = at - p.rotYf;
                float ph = (float)((double)b + kHalfPI);
                cph[m] = cos_f32(ph);
            }
            // SymmetryCosts row setup, Kernel.cu:292-299.
            double al = x * (double)rm.ux;
            al = al + y * (double)rm.uy;
            float sd = (float)(2.0 * (rm.along_f - al));
            rxs[m] = (float)(x + (double)(sd * rm.ux));
            rys[m] = (float)(y + (double)(sd * rm.uy));
            float rr = (float)(rm.two_focal_rot - op.ry[m]);
            if ((double)rr < -kPI) rr = (float)((double)rr + kTwoPI);
            rrs[m] = rr;
            // Off-limits box at the object's pose; SurfaceAreaCosts terms, Kernel.cu:469-480.
            const float4 box = shape_box(os, p.xf, p.yf);
            if constexpr (WITH_OL) stage(ch.OFF).put(i, box);
            sao[m] = comp_overlaps(rm, box);
            boxo[m] = box;
        }
        if constexpr (!SHARED) {
            if (!(MH_ABLATE & 16) && i < rm.r) rel_terms(ch, i, rpw[m], rang[m]);
        }
        if constexpr (NPL == 1) {
            clo.rpw = rpw[0];
            clo.rang = rang[0];
            clo.cph = cph[0];
            if constexpr (!SHARED) {
                clo.dc = clo.dr = false;
                clo.eang = 0.0f;
            }
        }
        if (i < c) {
            const RectShape cs = ch.clrs[i];
            const ObjP ps = ch.P[cs.pad];
            stage(ch.CLA).put(i, shape_box(cs, ps.xf, ps.yf));  // ClearanceCosts, :414-415
        }
        // SurfaceArea quirk: clearance i at object i's pose (cfg[i], :456). Steps with one
        // object per lane keep the overlaps unless object i moved, so most steps skip the pass.
        bool sa_new = i < c;
        if constexpr (SHARED) {
            sac[m] = clp.sac;
            sa_new = sa_new && (i == ka || i == kb);
        }
        if (sa_new) {
            const ObjP pi = ch.P[i];
            sac[m] = comp_overlaps(rm, shape_box(ch.clrs[i], pi.xf, pi.yf));
        }
        if constexpr (NPL == 1) clo.sac = sac[0];
    }
    }
    // Phase A's per-object terms and boxes: the Clearance pairs, OffLimits and the replay read
    // other lanes'.
    hand_off(ch.PX, ch.PY, ch.CLA, ch.OFF);

    // Phase B: symmetry rows, Kernel.cu:301-312. Row max over j of the reference's value,
    // which needs two correctly rounded square roots and ~25 fp64 operations per pair.
    // An fp32 estimate whose error is bounded by sym_err() screens the pairs; the reference's
    // formula is evaluated exactly only where the estimate cannot rule a pair out, and max is
    // exact, so the row maxima are the reference's bit for bit. A pose outside the range the
    // bound is proven for (exact_mode) evaluates every pair exactly.
    if (r == 0) MH_PHASE(ch, 1, t0);
    const bool exact_mode = group_ballot<L>(wild, gbase) != 0;
    // Steps that decide on the rejection bound leave a re-scanned row's maximum as its leader's
    // fp32 estimate (the bound adds its allowance, esym); the leader's exact value is evaluated
    // only if the step is not certainly rejected (below), when the row enters a commit or a sum.
    constexpr bool DEFER_SYM = FAST;  // (one chain per wavefront, one object per lane)
    int dlead = -1;
    float esym = 0.0f;
    if constexpr (!DELTA) {
    // Full scan: keep the two largest estimates per row and evaluate the leader exactly. When
    // the top two are closer than their error bounds the row falls back to the exact value of
    // every candidate within the bound.
    float m1[NPL], m2[NPL];
    int j1[NPL];
    for (int rep = 0; rep < MH_REPS(2); ++rep) {
    MH_CLOBBER();
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
        m1[m] = m2[m] = -INFINITY;
        j1[m] = -1;
    }
#pragma unroll 2
    for (int j = 0; j < ((MH_ABLATE & 1) ? 0 : n); ++j) {
        const float4 q = objp_f4(ch.P[j]);
#pragma unroll
        for (int m = 0; m < NPL; ++m) {
            const float v = sym_val_fast(q, rxs[m], rys[m], rrs[m]);
            m2[m] = __builtin_amdgcn_fmed3f(m1[m], m2[m], v);
            const bool up = v > m1[m];
            m1[m] = up ? v : m1[m];
            j1[m] = up ? j : j1[m];
        }
    }
    }
    bool amb[NPL];
    bool any_amb = false;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
        const int i = m * L + r;
        const bool row = i < n;
        const bool clear = j1[m] >= 0 &&
                           (m2[m] == -INFINITY ||
                            m1[m] - m2[m] > sym_err(m1[m], rrs[m]) + sym_err(m2[m], rrs[m]));
        amb[m] = row && (exact_mode || !clear);
        any_amb |= amb[m];
        float e = 0.0f;
        const double ry1 = pose_ry_var<L, NPL>(op, j1[m], gbase);  // (every lane active)
        if (row && j1[m] >= 0 && MH_CK(j1[m] < n, 7, j1[m], i)) {
            const ObjP q = ch.P[j1[m]];
            e = sym_val_exact(q.xf, q.yf, ry1, rxs[m], rys[m], (double)rrs[m]);
        }
        sym.mx[m] = fmaxf(0.0f, e);
        sym.arg[m] = e > 0.0f ? j1[m] : -1;
    }
    if (__ballot(any_amb)) {
        float thr[NPL];
#pragma unroll
        for (int m = 0; m < NPL; ++m) {
            thr[m] = (exact_mode || j1[m] < 0) ? INFINITY
                                               : 2.0f * sym_err(fabsf(m1[m]) + 1.0f, rrs[m]);
            if (amb[m]) {
                sym.mx[m] = 0.0f;
                sym.arg[m] = -1;
            }
        }
        for (int j = 0; j < n; ++j) {
            const ObjP q = ch.P[j];
            const double ryj = pose_ry<L, NPL>(op, j, gbase);
#pragma unroll
            for (int m = 0; m < NPL; ++m) {
                if (amb[m]) {
                    const float v = sym_val_fast(objp_f4(q), rxs[m],
                                                 rys[m], rrs[m]);
                    if (!(v < m1[m] - thr[m])) {
                        const float e = sym_val_exact(q.xf, q.yf, ryj, rxs[m], rys[m],
                                                      (double)rrs[m]);
                        if (e > sym.mx[m]) {
                            sym.mx[m] = e;
                            sym.arg[m] = j;
                        }
                    }
                }
            }
        }
    }
    } else {
    // PAIRS (the few-chains instance) with at most 8 objects: all N^2 pairs at once, lane
    // 8 i + j evaluating pair (i, j) exactly as the reference does, then each 8-lane group's
    // maximum (floored at 0, Kernel.cu:303-311; max is exact, so the order does not matter) and
    // its lowest column go to row i's owner lane. One exact evaluation on the step's critical
    // path instead of the screened passes below, which a wavefront per SIMD waits out in full.
    bool pairs_done = false;
    if constexpr (PAIRS && L == 64 && NPL == 1) {
        if (n <= 8) {
            const int pi = r >> 3, pj = r & 7;
            const int ai = pi << 2, aj = pj << 2;
            const float prx = __int_as_float(__builtin_amdgcn_ds_bpermute(ai, __float_as_int(rxs[0])));
            const float pry = __int_as_float(__builtin_amdgcn_ds_bpermute(ai, __float_as_int(rys[0])));
            const float prr = __int_as_float(__builtin_amdgcn_ds_bpermute(ai, __float_as_int(rrs[0])));
            const double ryj = __hiloint2double(__builtin_amdgcn_ds_bpermute(aj, __double2hiint(op.ry[0])),
                                                __builtin_amdgcn_ds_bpermute(aj, __double2loint(op.ry[0])));
            const ObjP q = ch.P[pj];
            float v = 0.0f;
            if (pi < n && pj < n)
                v = fmaxf(0.0f, sym_val_exact(q.xf, q.yf, ryj, prx, pry, (double)prr));
            int j = v > 0.0f ? pj : 8;
            group_max_arg<8>(v, j);
            const int src = (r & 7) << 5;  // lane 8 r holds row r's maximum
            const float mx = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(v)));
            const int ag = __builtin_amdgcn_ds_bpermute(src, j);
            sym.mx[0] = r < n ? mx : 0.0f;
            sym.arg[0] = (r < n && ag < 8) ? ag : -1;
            pairs_done = true;
        }
    }
    // Delta: only rows ka, kb and columns ka, kb changed. An unchanged row keeps its maximum
    // unless a changed column beats it (screened by the estimate) or its argmax column is a
    // changed one whose value dropped; changed rows and such rows are re-scanned by the whole
    // group, one row at a time.
    for (int rep = 0; rep < MH_REPS(64) && !pairs_done; ++rep) {
    MH_CLOBBER();
    bool need[NPL];
    unsigned pend[NPL];
    float4 qa = make_float4(0.f, 0.f, 0.f, 0.f), qb = qa;
    if (ka >= 0) qa = objp_f4(ch.P[ka]);
    if (kb >= 0) qb = objp_f4(ch.P[kb]);
    // the changed columns' rotY, from their owner lanes (ka, kb are group-uniform)
    const double rya = pose_ry<L, NPL>(op, ka < 0 ? 0 : ka, gbase);
    const double ryb = pose_ry<L, NPL>(op, kb < 0 ? 0 : kb, gbase);
    bool any_pend = false;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
        const int i = m * L + r;
        const bool row = i < n;
        const float cm = prev.mx[m];
        const int ca = prev.arg[m];
        sym.mx[m] = cm;
        sym.arg[m] = ca;
        need[m] = row && (i == ka || i == kb);
        pend[m] = 0u;
        if (row && !need[m]) {
            // A changed column's pair is pending (exact value needed) unless its estimate is
            // certainly below the old maximum; if that column held the maximum, the maximum
            // certainly dropped and the row is re-scanned without the exact value.
            if (ka >= 0) {
                const float v = sym_val_fast(qa, rxs[m], rys[m], rrs[m]);
                const bool below = !exact_mode && v + sym_err(v, rrs[m]) < cm;
                if (ca == ka && below) need[m] = true;
                else if (!below) pend[m] |= 1u;
            }
            if (kb >= 0) {
                const float v = sym_val_fast(qb, rxs[m], rys[m], rrs[m]);
                const bool below = !exact_mode && v + sym_err(v, rrs[m]) < cm;
                if (ca == kb && below) need[m] = true;
                else if (!below) pend[m] |= 2u;
            }
            if (need[m]) pend[m] = 0u;
        }
        any_pend |= pend[m] != 0u;
    }
    // Exact values of the pending (row, column) pairs: one evaluation site, each lane taking
    // its lowest pending slot per pass.
    while (__ballot(any_pend)) {
        if (any_pend) {
            int ms = NPL - 1;
#pragma unroll
            for (int m = NPL - 2; m >= 0; --m) ms = pend[m] ? m : ms;
            const unsigned pm = sel<NPL>(pend, ms);
            const int col = (pm & 1u) ? ka : kb;
            MH_CK(col >= 0 && col < n, 8, col, pm);
            const ObjP q = ch.P[col];
            const float e = sym_val_exact(q.xf, q.yf, (pm & 1u) ? rya : ryb, sel<NPL>(rxs, ms),
                                          sel<NPL>(rys, ms), (double)sel<NPL>(rrs, ms));
            any_pend = false;
#pragma unroll
            for (int m = 0; m < NPL; ++m) {
                if (m == ms) {
                    pend[m] &= pend[m] - 1u;
                    if (col == prev.arg[m] && !(e >= prev.mx[m])) {
                        need[m] = true;  // the old maximum is gone: re-scan the row
                    } else if (e > sym.mx[m]) {
                        sym.mx[m] = e;
                        sym.arg[m] = col;
                    }
                }
                any_pend |= pend[m] != 0u;
            }
        }
    }
    // Re-scans, one row at a time across the whole group: estimates and the top-2 reduction
    // here; the exact value of a clear row's leader is evaluated afterwards by the row's owner
    // lane, all rows in one pass.
    uint64_t rows[NPL];
    int lead[NPL];
    unsigned leadp = 0u;  // slots with a leader pending exact evaluation
#pragma unroll
    for (int m = 0; m < NPL; ++m) lead[m] = -1;
    bool any_row = false;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
        rows[m] = group_ballot<L>(need[m], gbase);
        any_row |= rows[m] != 0;
    }
    while (any_row) {
        int ms = NPL - 1;
#pragma unroll
        for (int m = NPL - 2; m >= 0; --m) ms = rows[m] ? m : ms;
        const uint64_t bm = sel<NPL>(rows, ms);
        const int b = __builtin_ctzll(bm);
        const float rx = grp_get<L>(sel<NPL>(rxs, ms), b, gbase);
        const float ry = grp_get<L>(sel<NPL>(rys, ms), b, gbase);
        const float rr = grp_get<L>(sel<NPL>(rrs, ms), b, gbase);
        float t1 = -INFINITY, t2 = -INFINITY;
        int tj = -1;
#pragma unroll
        for (int q = 0; q < NPL; ++q) {
            const int j = q * L + r;
            if (j < n) {
                const float v =
                    sym_val_fast(objp_f4(ch.P[j]), rx, ry, rr);
                t2 = __builtin_amdgcn_fmed3f(t1, t2, v);
                const bool up = v > t1;
                t1 = up ? v : t1;
                tj = up ? j : tj;
            }
        }
        const SymLead ld = group_sym_lead<L>(t1, t2, tj, r, gbase, rr);
        float best = 0.0f;
        int barg = -1;
        const bool clear = !exact_mode && ld.clear;
        if (!clear) {
            const float thr =
                (exact_mode || ld.j < 0) ? INFINITY : 2.0f * sym_err(fabsf(ld.m) + 1.0f, rr);
            float bv = -INFINITY;
            int bj = -1;
#pragma unroll
            for (int q = 0; q < NPL; ++q) {  // this lane's columns j = q * L + r
                const int j = q * L + r;
                if (j >= n) break;
                const ObjP p = ch.P[j];
                const float v = sym_val_fast(objp_f4(p), rx, ry, rr);
                if (!(v < ld.m - thr)) {
                    const float e = sym_val_exact(p.xf, p.yf, op.ry[q], rx, ry, (double)rr);
                    if (e > bv) {
                        bv = e;
                        bj = j;
                    }
                }
            }
            group_max_arg<L>(bv, bj);
            best = bv > 0.0f ? bv : 0.0f;
            barg = bv > 0.0f ? bj : -1;
        }
        any_row = false;
#pragma unroll
        for (int m = 0; m < NPL; ++m) {
            if (m == ms) {
                if (r == b) {
                    if (clear && DEFER_SYM) {
                        dlead = ld.j;
                        esym = sym_err(ld.m, rr);
                        sym.mx[m] = fmaxf(0.0f, ld.m);
                    } else if (clear) {
                        lead[m] = ld.j;
                        leadp |= 1u << m;
                    } else {
                        sym.mx[m] = best;
                        sym.arg[m] = barg;
                    }
                }
                rows[m] &= rows[m] - 1;
            }
            any_row |= rows[m] != 0;
        }
    }
    while (__ballot(leadp != 0u)) {
        const int ms = leadp ? __builtin_ctz(leadp) : 0;
        const int j = leadp ? sel<NPL>(lead, ms) : 0;
        const double ryj = pose_ry_var<L, NPL>(op, j, gbase);  // (every lane active)
        if (leadp) {
            leadp &= leadp - 1u;
            MH_CK(j >= 0 && j < n, 9, j, ms);
            const ObjP q = ch.P[j];
            const float e = sym_val_exact(q.xf, q.yf, ryj, sel<NPL>(rxs, ms),
                                          sel<NPL>(rys, ms), (double)sel<NPL>(rrs, ms));
#pragma unroll
            for (int m = 0; m < NPL; ++m) {
                if (m == ms) {
                    sym.mx[m] = fmaxf(0.0f, e);
                    sym.arg[m] = e > 0.0f ? j : -1;
                }
            }
        }
    }
    }
    }

    if (r == 0) MH_PHASE(ch, 2, t0);
    // One object per lane: the non-zero Clearance pairs are tracked incrementally
    // (inc_cl_update); the 8-lane instance keeps the direct pass below (with a handful of
    // clearances its latency is lower, and those rooms run few chains).
    constexpr bool INC_CL = DELTA && NPL == 1 && L >= 16;
    int cl_total = 0;
    // (a lane's column of Clearance pairs changes when its object moved or a moved clearance
    // pairs with it before or after)
    bool colchg = r < n && (r == ka || r == kb);
    if constexpr (INC_CL) {
#if MH_DOUBLE & 128
        const bool colchg0 = colchg;
        for (int rep = 0; rep < 2; ++rep) {
            MH_CLOBBER();
            colchg = colchg0;
#endif
            cl_total = inc_cl_update<L>(ch, n, c, ka, kb, r, gbase, boxo[0], clp, clo, colchg);
#if MH_DOUBLE & 128
        }
#endif
    }
    if (r == 0) MH_PHASE(ch, 3, t0);
    if constexpr (FAST) {
        static_assert(INC_CL && L == 64, "the rejection bound needs one chain per wavefront");
        if (rm.r <= L) {  // every relationship term is held by a lane (rpw[0], rang[0])
            // this lane's object against the clearances it overlaps: kept from the current
            // configuration unless its column may have changed
            int d = BOUND_OPEN;
#if MH_DOUBLE & 256
            for (int rep = 0; rep < 2; ++rep) {
            MH_CLOBBER();
            float px0 = px[0];
            asm volatile("" : "+v"(px0));  // (the probe's second pass is not folded into the first)
#else
            const float px0 = px[0];
#endif
            float clsum = clp.clc;
            uint64_t bits = r < n ? clo.cm : 0ull;
            const int kcl = __builtin_popcountll(bits);
            if (__ballot(colchg)) {
                if (colchg) {
                    clsum = 0.0f;
                    while (bits) {
                        const int i = __builtin_ctzll(bits);
                        bits &= bits - 1;
                        clsum += overlap(ch.CLA[i], boxo[0]);
                    }
                }
            }
            clo.clc = clsum;
#if MH_CHECK
            {  // the cached column sum against a fresh one
                float f = 0.0f;
                uint64_t b2 = r < n ? clo.cm : 0ull;
                while (b2) {
                    const int i = __builtin_ctzll(b2);
                    b2 &= b2 - 1;
                    f += overlap(ch.CLA[i], boxo[0]);
                }
                MH_CK(f == clsum, 28, __float_as_uint(f), __float_as_uint(clsum));
            }
#endif
            BoundTerms bt;
            bt.nx = px0;
            bt.ny = py[0];
            bt.anx = fabsf(bt.nx);
            bt.any = fabsf(bt.ny);
            bt.fp = -cph[0];
            bt.afp = fabsf(bt.fp);
            bt.sym = -sym.mx[0];
            bt.symw = r < n ? (float)(n - r) * (sym.mx[0] + esym) : 0.0f;  // (row r: position r)
            bt.esym = esym;
            bt.cl = -clsum;
            bt.kcl = kcl;
            bt.clpos = 0.0f;  // (no position credit: the list positions are not formed here)
            bt.pwd = bt.angd = 0.0;
            bt.efp = r < n && clo.dc ? kDeltaCph : 0.0f;  // (fp32 estimates, approx_terms)
            bt.eang = r < rm.r && clo.dr ? clo.eang : 0.0f;
            bt.pwx = __ballot(r < rm.r && clo.dr) ? kPwEstU : 0;
            bt.sa = -((sac[0].x + sac[0].y + sac[0].z + sac[0].w) +
                      (sao[0].x + sao[0].y + sao[0].z + sao[0].w));
            bt.pw = -(float)rpw[0];
            bt.ang = -(float)rang[0];
            bt.aang = fabsf(bt.ang);
            bt.k = 8;  // the SurfaceArea partial sum adds eight overlaps
            d = bound_decide(rm, n, c, rm.r, cl_total, bt, u_acc, cur, *star_iv, a.bound_slack);
#if MH_DOUBLE & 256
            }
#endif
            if (r == 0) MH_PHASE(ch, 4, t0);
#if MH_STAMPS
            if (r == 0) {
                stage(ch.aux)->cyc[8] += 1;
                stage(ch.aux)->cyc[9] += d == BOUND_REJECT ? 1 : 0;
                stage(ch.aux)->cyc[10] += d == BOUND_ACCEPT ? 1 : 0;
            }
#endif
            if (d == BOUND_REJECT) {
                *fast = d;
                return;
            }
            if constexpr (DEFER_SYM) {
                // the deferred leaders' exact values (every lane active for the rotY read)
                if (__ballot(dlead >= 0)) {
                    const int j = dlead >= 0 ? dlead : 0;
                    const double ryj = pose_ry_var<L, NPL>(op, j, gbase);
                    if (dlead >= 0) {
                        const ObjP q = ch.P[j];
                        const float e = sym_val_exact(q.xf, q.yf, ryj, rxs[0], rys[0],
                                                      (double)rrs[0]);
                        MH_CK(fabsf(fmaxf(0.0f, e) - sym.mx[0]) <= esym, 33,
                              __float_as_uint(e), __float_as_uint(sym.mx[0]));
                        sym.mx[0] = fmaxf(0.0f, e);
                        sym.arg[0] = e > 0.0f ? j : -1;
                    }
                }
                if (d != BOUND_OPEN) {
                    *fast = d;
                    return;
                }
            }
            // The exact sums are needed: every estimated term is made exact first.
            const bool obj = r < n && clo.dc, rel = r < rm.r && clo.dr;
            if (__ballot(obj || rel)) {
                float c0 = cph[0];
                double p0 = rpw[0], a0 = rang[0];
                exact_terms(ch, rm, r, n, obj, rel, c0, p0, a0);
#if MH_CHECK
                // the estimates' allowances, against the exact values
                MH_CK(!obj || fabsf(cph[0] - c0) <= kDeltaCph, 30, __float_as_uint(cph[0]),
                      __float_as_uint(c0));
                MH_CK(!rel || fabs(rpw[0] - p0) <= kPwEstU * 0x1p-24 * fabs(p0) + 1e-30, 31,
                      __float_as_uint((float)rpw[0]), __float_as_uint((float)p0));
                MH_CK(!rel || fabs(rang[0] - a0) <= (double)clo.eang, 32,
                      __float_as_uint((float)rang[0]), __float_as_uint((float)a0));
#endif
                cph[0] = c0;
                rpw[0] = p0;
                rang[0] = a0;
                clo.cph = c0;
                clo.rpw = p0;
                clo.rang = a0;
            }
            clo.dc = clo.dr = false;
            clo.eang = 0.0f;
        }
    }
    // The eight ordered sums of Costs() -- VisualBalance nx and ny (float through double
    // temporaries, :200-201), FocalPoint (double, :277), Symmetry (float, :314), SurfaceArea
    // (float, :463-479), Clearance (float, :429), PairWise and PairWiseAngle (double, :222,
    // :249/253) -- are replayed in the reference's order by lanes 0..7 of the group at once,
    // from per-object values (dense) and compacted lists of the non-zero sparse terms
    // (x - 0 == x, so dropping exact zeros is exact). Each step is rn_d(acc + v) with v the
    // negated term where the reference subtracts, rounded on to float for the float
    // accumulators (rn_f(rn_d(a + b)) == rn_f(a + b) for floats: 53 >= 2*24 + 2 bits).
    double acc = 0.0;  // lane k of the group owns sum k (k = 5 unused; SurfaceArea below)
    const bool acc_float = (r == 0 || r == 1 || r == 3 || r == 4);
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
        const int i = m * L + r;
        if (i < n) {
            stage(ch.CPHF).put(i, -cph[m]);
            stage(ch.RMXF).put(i, -sym.mx[m]);
        }
    }
    // SurfaceAreaCosts: clearances (quirk box at cfg[i]) first, then objects (:453-480);
    // its terms are almost always all zero, so the group walks the non-zero ones directly.
    float sa = 0.0f;
    for (int rep = 0; rep < MH_REPS(4); ++rep) {
    MH_CLOBBER();
    sa = 0.0f;
#pragma unroll
    for (int m = 0; m < NPL; ++m)
        if (m * L < c) sa = serial_sub4<L>(sa, sac[m], gbase);
#pragma unroll
    for (int m = 0; m < NPL; ++m)
        if (m * L < n) sa = serial_sub4<L>(sa, sao[m], gbase);
    }

    // ClearanceCosts pairs, clearance-major then object (Kernel.cu:408-431).
    int cnt_cl = 0;
    // One object per lane: only the non-zero pairs (inc_cl_update) are re-evaluated, each by its
    // object's lane, and written straight to their list positions (row prefix + the row's set
    // bits below the object).
    constexpr bool CL_STATE = NPL == 1 && L >= 16;  // pair state kept for the steps
    bool cl_done = false;
    if constexpr (NPL == 1) {
        const int j = r;
        const float4 boxj = boxo[0];
        if constexpr (INC_CL) {
            const uint64_t* NZn = ch.NZ.ptr() + clo.buf * c;
            if (cl_total <= 2 * L) {  // fits the list: write every term at its position
                const uint64_t below = (1ull << j) - 1ull;
                uint64_t bits = j < n ? clo.cm : 0ull;
                while (bits) {
                    const int i = __builtin_ctzll(bits);
                    bits &= bits - 1;
                    const int pos = ch.PRE[i] + __builtin_popcountll(NZn[i] & below);
                    if (MH_CK(i < c && pos >= 0 && pos < 2 * L, 6, i, pos))
                        stage(ch.LCL).put(pos, (double)-overlap(ch.CLA[i], boxj));
                }
                cnt_cl = cl_total;
                cl_done = true;
            }
        } else if constexpr (!DELTA && CL_STATE) {
            // full evaluation: the pair state from scratch, for the steps that follow
            uint64_t cm = 0ull;
            float clc = 0.0f;
            for (int i = 0; i < c; ++i) {
                const float ov = j < n ? overlap(ch.CLA[i], boxj) : 0.0f;
                const bool nzi = ov != 0.0f;
                const uint64_t row = group_ballot<L>(nzi, gbase);
                cm |= (uint64_t)nzi << i;
                if (nzi) clc += ov;
                if (r == 0) stage(ch.NZ).put(i, row);
            }
            clo.cm = cm;
            clo.buf = 0;
            clo.clc = clc;
        }
    }
    for (int rep = 0; rep < MH_REPS(8); ++rep) {
    if (cl_done) break;
    MH_CLOBBER();
    cnt_cl = 0;
    float4 offb[NPL];
#pragma unroll
    for (int m = 0; m < NPL; ++m) {  // this lane's off-limits boxes (recomputed: no LDS copy)
        const int j = m * L + r;
        offb[m] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (j < n) {
            const ObjP p = ch.P[j];
            offb[m] = shape_box(ch.objs[j], p.xf, p.yf);
        }
    }
    const int cend = (MH_ABLATE & 8) ? 0 : c;
    // One object per lane: two clearances per iteration (boxes for the next two in flight),
    // one overflow test and count update per pair (a pair appends at most 2L <= capacity
    // terms). Otherwise one clearance per iteration.
    float4 A0n = cend > 0 ? ch.CLA[0] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 A1n = cend > 1 ? ch.CLA[1] : make_float4(0.f, 0.f, 0.f, 0.f);
    int ci = 0;
    for (; NPL == 1 && ci + 1 < cend; ci += 2) {
        const float4 A0 = A0n, A1 = A1n;
        if (ci + 2 < cend) A0n = ch.CLA[ci + 2];
        if (ci + 3 < cend) A1n = ch.CLA[ci + 3];
        double v[2 * NPL];
        bool nz[2 * NPL];
#pragma unroll
        for (int m = 0; m < NPL; ++m) {
            const bool own = m * L + r < n;
            const float a0 = own ? overlap(A0, offb[m]) : 0.0f;
            const float a1 = own ? overlap(A1, offb[m]) : 0.0f;
            v[m] = (double)-a0;
            nz[m] = a0 != 0.0f;
            v[NPL + m] = (double)-a1;
            nz[NPL + m] = a1 != 0.0f;
        }
        list_append_n<L, 2 * NPL, double>(stage(ch.LCL), 2 * L, cnt_cl, acc, r == 4, true, v, nz,
                                          r, gbase);
    }
    for (; ci < cend; ++ci) {
        const float4 A = A0n;  // box ci; box ci + 1 is in flight during the appends
        if (ci + 1 < cend) A0n = ch.CLA[ci + 1];
#pragma unroll
        for (int m = 0; m < NPL; ++m) {
            const int j = m * L + r;
            const float ar = (j < n) ? overlap(A, offb[m]) : 0.0f;
            list_append<L, double>(stage(ch.LCL), 2 * L, cnt_cl, acc, r == 4, true, (double)-ar,
                                   ar != 0.0f, r, gbase);
        }
    }
    }

    if (r == 0) MH_PHASE(ch, 5, t0);  // SurfaceArea walk and Clearance list
    // PairWiseCosts (:210-233) and PairWiseAngleCosts (:236-263) terms.
    int cnt_pw = 0, cnt_ang = 0;
    for (int rep = 0; rep < MH_REPS(16); ++rep) {
    MH_CLOBBER();
    cnt_pw = cnt_ang = 0;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
        if (m * L >= rm.r) break;
        list_append<L, double>(stage(ch.LPW), ch.lst_r, cnt_pw, acc, r == 6, false, -rpw[m],
                               rpw[m] != 0.0, r, gbase);
        list_append<L, double>(stage(ch.LANG), ch.lst_r, cnt_ang, acc, r == 7, false, -rang[m],
                               rang[m] != 0.0, r, gbase);
    }
    for (int qb = NPL * L; qb < ((MH_ABLATE & 16) ? 0 : rm.r); qb += L) {  // R > L * NPL
        const int q = qb + r;
        double tpw = 0.0, tang = 0.0;
        if (q < rm.r) rel_terms(ch, q, tpw, tang);
        list_append<L, double>(stage(ch.LPW), ch.lst_r, cnt_pw, acc, r == 6, false, -tpw,
                               tpw != 0.0, r, gbase);
        list_append<L, double>(stage(ch.LANG), ch.lst_r, cnt_ang, acc, r == 7, false, -tang,
                               tang != 0.0, r, gbase);
    }
    }

    // The replay: lane k walks its own sequence in the reference's order. Lanes 0/1: the
    // VisualBalance products (double terms, float accumulators); 2: -cos phi (float terms,
    // double accumulator); 3: -row max (float, float); 4: Clearance list (float, float);
    // 6/7: PairWise / Angle lists (double, double). Every sequence is zero-padded to a multiple
    // of four terms; a lane reads four at a time (two ds_read_b128 of doubles or one of
    // floats) and keeps both a double- and a float-rounded walk of the same terms.
    for (int q = cnt_cl + r; q < ((cnt_cl + 3) & ~3); q += L) stage(ch.LCL).put(q, 0.0);
    for (int q = cnt_pw + r; q < ((cnt_pw + 3) & ~3); q += L) stage(ch.LPW).put(q, 0.0);
    for (int q = cnt_ang + r; q < ((cnt_ang + 3) & ~3); q += L) stage(ch.LANG).put(q, 0.0);
    // the replay's streams, as their lanes walk them
    hand_off(ch.CPHF, ch.RMXF, ch.LCL, ch.LPW, ch.LANG);
    const double acc0 = acc;
    for (int rep = 0; rep < MH_REPS(32); ++rep) {
        MH_CLOBBER();
        const int k = r;
        const double* dsrc = ch.zero4;
        int len = 0;
        if (k == 0 || k == 1) {
            dsrc = k == 0 ? ch.PX.ptr() : ch.PY.ptr();
            len = n;
        } else if (k == 2 || k == 3) {
            dsrc = k == 2 ? ch.CPHF.ptr() : ch.RMXF.ptr();
            len = n;
        } else if (k == 4) {
            dsrc = ch.LCL.ptr();
            len = cnt_cl;
        } else if (k == 6 || k == 7) {
            dsrc = k == 6 ? ch.LPW.ptr() : ch.LANG.ptr();
            len = k == 6 ? cnt_pw : cnt_ang;
        }
        len = (len + 3) & ~3;
        // The Clearance list (float terms, float accumulator) usually outruns the dense sums:
        // its part past them runs in plain fp32 below (rn_f(a + b) is the reference's float add).
        // The walk's length comes from the group-uniform counts, with no cross-lane reduction.
        const int steps = max(a.lay.N4, max((cnt_pw + 3) & ~3, (cnt_ang + 3) & ~3));
        double accd = acc0, accf = acc0;
        for (int l0 = 0; l0 < steps; l0 += 4) {
            // every stream holds doubles; a lane past its end reads four zeros
            const double* src = l0 < len ? dsrc + l0 : ch.zero4;
            const double2 a0 = load16<double2>(src);
            const double2 a1 = load16<double2>(src + 2);
            const double v[4] = {a0.x, a0.y, a1.x, a1.y};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                accd = accd + v[u];
                accf = (double)(float)(accf + v[u]);
            }
        }
        if (k == 4 && len > steps) {
            float a32 = (float)accf;
            for (int l0 = steps; l0 < len; l0 += 4) {
                const double2 a0 = load16<double2>(dsrc + l0);
                const double2 a1 = load16<double2>(dsrc + l0 + 2);
                a32 = a32 + (float)a0.x;
                a32 = a32 + (float)a0.y;
                a32 = a32 + (float)a1.x;
                a32 = a32 + (float)a1.y;
            }
            accf = a32;
        }
        acc = acc_float ? accf : accd;
    }
    const float nx = (float)grp_get<L>(acc, 0, gbase);
    const float ny = (float)grp_get<L>(acc, 1, gbase);
    const double fp = grp_get<L>(acc, 2, gbase);
    const float symc = (float)grp_get<L>(acc, 3, gbase);
    const float cl = (float)grp_get<L>(acc, 4, gbase);
    const double pw = grp_get<L>(acc, 6, gbase);
    const double ang = grp_get<L>(acc, 7, gbase);
    // (the replay's reads are done before a lane rewrites its streams)
    hand_off(ch.PX, ch.PY, ch.CPHF, ch.RMXF, ch.LCL, ch.LPW, ch.LANG);
    const float vb = (float)(-1.0 * distance_f(nx / rm.denom, ny / rm.denom, rm.cxf, rm.cyf));

    if (r == 0) MH_PHASE(ch, 6, t0);
    // OffLimitsCosts, pairs i < j (Kernel.cu:488-511): final / evaluation passes only.
    float ol = 0.0f;
    if constexpr (WITH_OL) {
        for (int i = 0; i < n; ++i) {
            const float4 A = ch.OFF[i];
            for (int jb = i + 1; jb < n; jb += L) {
                const int j = jb + r;
                const float ar = (j < n) ? overlap(A, ch.OFF[j]) : 0.0f;
                ol = serial_sub<L>(ol, ar, gbase);
            }
        }
    }

    // Costs(), Kernel.cu:518-549.
    const float pwc = (float)(pw * ang);
    out[1] = rm.w_pw * pwc;
    out[2] = rm.w_vb * vb;
    out[3] = rm.w_fp * (float)fp;
    out[4] = rm.w_sym * symc;
    out[6] = rm.w_ol * ol;
    out[5] = rm.w_cl * cl;
    out[7] = rm.w_sa * sa;
    float t = out[1] + out[2];
    t = t + out[3];
    t = t + out[4];
    t = t + out[5];
    t = t + out[7];
    out[0] = t;
    if (save && r == 0)  // (the caller then keeps only the total in a register)
        for (int k = 0; k < 8; ++k) stage(ch.aux)->star[k] = out[k];
}

// ---- propose(), Kernel.cu:566-704, applied in place --------------------------------------

// Object k's pose (k group-uniform), from its owner lane.
template <int L, int NPL>
__device__ __forceinline__ Backup read_obj(const OwnPose<NPL>& op, int k, int gbase) {
    Backup b;
    b.k = k;
    const int m = k / L, src = k % L;
    b.x = grp_get<L>(sel<NPL>(op.x, m), src, gbase);
    b.y = grp_get<L>(sel<NPL>(op.y, m), src, gbase);
    b.ry = grp_get<L>(sel<NPL>(op.ry, m), src, gbase);
    return b;
}

// Sets object k's pose (group-uniform k and values): its owner lane's registers, and the float
// pose words in LDS (`writer`).
template <int L, int NPL>
__device__ __forceinline__ void write_obj(const ChainPtrs& ch, OwnPose<NPL>& op, int r,
                                          bool writer, int k, double x, double y, double ry) {
    const bool own = r == k % L;
    const int km = k / L;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
        const bool here = own && m == km;
        op.x[m] = here ? x : op.x[m];
        op.y[m] = here ? y : op.y[m];
        op.ry[m] = here ? ry : op.ry[m];
    }
    if (writer && MH_CK(k >= 0 && k < ch.rm->n, 4, k, 0)) {
        ObjP p;
        p.xf = (float)x;
        p.yf = (float)y;
        p.rotYf = (float)ry;
        p.pad = 0.0f;
        stage(ch.P).put(k, p);
    }
}

// Applies one proposal to the configuration (registers and LDS); `writer` also records the
// overwritten objects in ch.aux so a rejection can undo them. Returns the objects it changed
// (-1: none).
template <int L, int NPL, class Rng>
__device__ MH_EVAL_ATTR int2 propose(Rng& rng, const DevRoom& rm, const unsigned char* frozen,
                        const ChainPtrs& ch, OwnPose<NPL>& op, int r, int gbase, bool writer) {
    const int n = rm.n;
    const int mode = rand_int(rng, 2, 0);
    if (mode == 0) {  // translate, Kernel.cu:595-632
        const int k = pick_object(rng, n, frozen);
        float dx = rng.normal();
        dx = dx * rm.sx;
        float dy = rng.normal();
        dy = dy * rm.sy;
        const Backup b0 = read_obj<L, NPL>(op, k, gbase);
        double x = b0.x, y = b0.y;
        if (x + (double)dx > rm.rmax_x) x = rm.rmax_x;
        else if (x + (double)dx < rm.rmin_x) x = rm.rmin_x;
        else x = x + (double)dx;
        if (y + (double)dy > rm.rmax_y) y = rm.rmax_y;
        else if (y + (double)dy < rm.rmin_y) y = rm.rmin_y;
        else y = y + (double)dy;
        if (writer) {
            const Staged<ChainAux> ax = stage(ch.aux);
            ax->b[0] = b0;
            ax->nb = 1;
            ax->swap_a = -1;
        }
        write_obj<L, NPL>(ch, op, r, writer, k, x, y, b0.ry);
        return make_int2(k, -1);
    }
    if (mode == 1) {  // rotate, Kernel.cu:634-653
        const int k = pick_object(rng, n, frozen);
        float dr = rng.normal();
        dr = (float)((double)dr * kSigmaT);
        const Backup b0 = read_obj<L, NPL>(op, k, gbase);
        double ry = b0.ry + (double)dr;
        if (ry < 0) ry = ry + kTwoPI;
        else if (ry > kTwoPI) ry = ry - kTwoPI;
        if (writer) {
            const Staged<ChainAux> ax = stage(ch.aux);
            ax->b[0] = b0;
            ax->nb = 1;
            ax->swap_a = -1;
        }
        write_obj<L, NPL>(ch, op, r, writer, k, b0.x, b0.y, ry);
        return make_int2(k, -1);
    }
    // swap, Kernel.cu:655-703: object 1's pose travels through float temporaries.
    if (n < 2) {
        if (writer) {
            const Staged<ChainAux> ax = stage(ch.aux);
            ax->nb = 0;
            ax->swap_a = -1;
        }
        return make_int2(-1, -1);
    }
    const int ka = pick_object(rng, n, frozen);
    const int kb = pick_object(rng, n, frozen);
    const Backup b0 = read_obj<L, NPL>(op, ka, gbase);
    const Backup b1 = read_obj<L, NPL>(op, kb, gbase);
    if (writer) {
        const Staged<ChainAux> ax = stage(ch.aux);
        ax->b[0] = b0;
        ax->b[1] = b1;
        ax->nb = 2;
        ax->swap_a = ka;
        ax->swap_b = kb;
    }
    write_obj<L, NPL>(ch, op, r, writer, ka, b1.x, b1.y, b1.ry);
    write_obj<L, NPL>(ch, op, r, writer, kb, (double)(float)b0.x, (double)(float)b0.y,
                      (double)(float)b0.ry);
    return make_int2(ka, kb == ka ? -1 : kb);
}

// Saves the proposed configuration as the chain's best (cfgStar, Kernel.cu:810-811): lane r
// writes its objects' x, y, rotY from registers; z, rotX, rotZ come from HBM with a pending swap
// applied as commit_swap_zrr would (ka takes kb's values, kb takes ka's rounded to float).
template <int L, int NPL>
__device__ __forceinline__ void save_best_pose(const ChainPtrs& ch, const OwnPose<NPL>& op,
                                               double* dst, int n, int r) {
    const int ka = ch.aux->swap_a, kb = ch.aux->swap_b;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
        const int i = m * L + r;
        if (i >= n) break;
        dst[F_X * n + i] = op.x[m];
        dst[F_Y * n + i] = op.y[m];
        dst[F_RY * n + i] = op.ry[m];
        int src = i;
        bool rnd = false;
        if (ka >= 0) {
            if (i == kb) {
                src = ka;
                rnd = true;
            } else if (i == ka) {
                src = kb;
            }
        }
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            const double v = ch.zrr[f * n + src];
            dst[(F_Z + f) * n + i] = rnd ? (double)(float)v : v;
        }
    }
}

// An accepted swap also exchanges z, rotX and rotZ (Kernel.cu:675-700), which no cost reads:
// they stay in HBM and are swapped there, object 1's values through float temporaries.
__device__ __forceinline__ void commit_swap_zrr(const ChainPtrs& ch, int n) {
    const int ka = ch.aux->swap_a, kb = ch.aux->swap_b;
    if (ka < 0) return;
    if (!MH_CK(ka < n && kb >= 0 && kb < n, 1, ka, kb)) return;
#pragma unroll
    for (int f = 0; f < 3; ++f) {
        double* row = ch.zrr + f * n;
        const double va = row[ka], vb = row[kb];
        row[ka] = vb;
        row[kb] = (double)(float)va;
    }
}

// Undo the last proposal (every lane of the group; the backups are group-uniform LDS reads),
// knowing which objects it changed (kk, as propose returned it: a swap of an object with itself
// restores only b[0], which holds the same original pose as b[1]). Both backups are read at once
// instead of after the count (config 3 114.5 -> 113.8 ms, config 2 4.24 -> 4.20 ms per launch).
template <int L, int NPL>
__device__ __forceinline__ void restore(const ChainPtrs& ch, OwnPose<NPL>& op, int r,
                                        bool writer, int2 kk) {
    const Backup b1 = ch.aux->b[1];
    const Backup b0 = ch.aux->b[0];
    if (kk.y >= 0 && MH_CK(b1.k == kk.y, 3, b1.k, kk.y))
        write_obj<L, NPL>(ch, op, r, writer, b1.k, b1.x, b1.y, b1.ry);
    if (kk.x >= 0 && MH_CK(b0.k == kk.x, 2, b0.k, kk.x))
        write_obj<L, NPL>(ch, op, r, writer, b0.k, b0.x, b0.y, b0.ry);
}

// ---- the kernel ---------------------------------------------------------------------------

// Steps of plain chains decide on the rejection bound when a chain owns the wavefront with one
// object per lane.
#define FASTK_OF(L, NPL) ((NPL) == 1 && (L) == 64 && !(MH_ABLATE & 4))

// Waves per SIMD the register allocator must leave room for. The plain step kernel with one
// chain per wavefront and one object per lane (config 3) is held to 5: its LDS then admits five
// 4-wave workgroups per CU, and 20 resident chains measured 4.47e8 chain-steps/s against 4.20e8
// with 16 (101 VGPRs). Other instances keep the allocator's choice, among them OP_STEP_FEW, the
// same step for launches of at most two chains per SIMD: at config 2 (N = 8, 1,024 chains, one
// wavefront per SIMD) the cap's spills and reloads sit on the critical path, and the uncapped
// build (122 VGPRs, no scratch) ran 1.92e8 chain-steps/s against 1.77e8 (gpurun_out/ab8a).
// $MH_WAVES_PER_EU builds
// (tools/build_ablate.sh wpeK) pin every instance for experiments.
template <int L, int NPL, int OP>
struct StepWaves {
#ifdef MH_WAVES_PER_EU
    static constexpr int value = MH_WAVES_PER_EU;
#else
    static constexpr int value = (L == 64 && NPL == 1 && OP == OP_STEP) ? 5 : 1;
#endif
};
#define MH_OCC __attribute__((amdgpu_waves_per_eu(StepWaves<L, NPL, OP>::value, 8)))

// Output slot of a chain: with parallel tempering the replica at rung k of group g goes to
// g*K + k (a session's chain offset and count are multiples of K).
__device__ __forceinline__ int64_t out_index(const LaunchArgs& a, int64_t chain) {
    if (a.n_temps <= 1) return chain;
    return chain - chain % a.n_temps + a.meta[chain].rung;
}

template <int L, int NPL, int OP>
__global__ void __launch_bounds__(512) MH_OCC mh_kernel(LaunchArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    // OP_STEP_T: OP_STEP with best-of-chain tracking compiled in; OP_STEP_XW: the same drawing
    // from the cuRAND XORWOW stream instead of Philox. Plain OP_STEP carries no tracking code.
    constexpr bool STEP =
        (OP == OP_STEP || OP == OP_STEP_T || OP == OP_STEP_XW || OP == OP_STEP_FEW);
    constexpr bool TRACK = (OP == OP_STEP_T || OP == OP_STEP_XW);
    // (one chain per wave draws from the wave-batched Philox window, its Box-Muller pairs in LDS)
    using Rng = typename std::conditional<OP != OP_STEP_XW && L == 64, WaveRngLds,
                                          typename RngOf<OP == OP_STEP_XW, L>::type>::type;
    constexpr int G = 64 / L;
    const int n = a.rm.n;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = (L == 64) ? 0 : lane / L;
    const int r = (L == 64) ? lane : lane % L;
    const int gbase = g * L;
    const int waves_per_wg = blockDim.x >> 6;

    // Room tables: staged once per workgroup (the chain loop then never touches global memory).
    constexpr FixedLds F = fixed_lds(L, NPL);  // compile-time part of the layout
    RectShape* objs_l = reinterpret_cast<RectShape*>(lds + F.h_obj);
    RectShape* clrs_l = reinterpret_cast<RectShape*>(lds + F.h_clr);
    RelConst* relc_l = reinterpret_cast<RelConst*>(lds + a.lay.h_rel);
    unsigned char* frozen = lds + F.h_frz;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        RectShape s = a.objc[i].off;
        s.pad = __float_as_int(a.objc[i].area);
        objs_l[i] = s;
    }
    for (int i = threadIdx.x; i < a.rm.c; i += blockDim.x) {
        RectShape s = a.clrc[i].shape;
        s.pad = a.clrc[i].src;
        clrs_l[i] = s;
    }
    uint2* rix_l = reinterpret_cast<uint2*>(lds + a.lay.h_rix);
    float4* re0_l = reinterpret_cast<float4*>(lds + a.lay.h_re);
    float4* re1_l = re0_l + (a.rm.r > 0 ? a.rm.r : 1);
    for (int i = threadIdx.x; i < a.rm.r; i += blockDim.x) {
        const RelConst rc = a.relc[i];
        relc_l[i] = rc;
        rix_l[i] = make_uint2((unsigned)rc.s | ((unsigned)rc.t << 16),
                              (unsigned)rc.as | ((unsigned)rc.at << 16));
        rel_est_consts(rc, re0_l[i], re1_l[i]);
    }
    for (int i = threadIdx.x; i <= n; i += blockDim.x) frozen[i] = (i < n) ? (a.objc[i].frozen != 0) : 1;
    DevRoom* rm_l = reinterpret_cast<DevRoom*>(lds + F.h_room);
    if (threadIdx.x == 0) *rm_l = a.rm;
    if (threadIdx.x < 4) reinterpret_cast<double*>(lds + F.h_zero)[threadIdx.x] = 0.0;
    __syncthreads();

    const int64_t chain = ((int64_t)blockIdx.x * waves_per_wg + wave) * G + g;
    if (chain >= a.n_chains) return;
    // (debug builds: the host's layout agrees with the compile-time one and fits the launch)
    MH_CK(a.lay.AUX == F.AUX && a.lay.PX == F.PX && a.lay.LCL == F.LCL && a.lay.stride >= F.end &&
              a.lay.hdr >= F.h_clr,
          13, a.lay.AUX, F.AUX);

    unsigned char* base = lds + a.lay.hdr + (wave * G + g) * a.lay.stride;
    ChainPtrs ch;
    ch.objs = objs_l;
    ch.clrs = clrs_l;
    ch.relc = relc_l;
    ch.rix = rix_l;
    ch.re0 = re0_l;
    ch.re1 = re1_l;
    ch.P = {reinterpret_cast<ObjP*>(base + F.P)};
    ch.PX = {reinterpret_cast<double*>(base + F.PX)};
    ch.PY = {reinterpret_cast<double*>(base + F.PY)};
    ch.CPHF = {reinterpret_cast<double*>(base + F.CPHF)};
    ch.RMXF = {reinterpret_cast<double*>(base + F.RMXF)};
    ch.LCL = {reinterpret_cast<double*>(base + F.LCL)};
    ch.LPW = {reinterpret_cast<double*>(base + a.lay.LPW)};
    ch.lst_r = a.lay.lst_r;
    ch.LANG = {reinterpret_cast<double*>(base + a.lay.LANG)};
    ch.zrr = a.st + chain * (int64_t)(F_COUNT * n) + F_Z * n;
    ch.OFF = {reinterpret_cast<float4*>(base + (a.lay.OFF >= 0 ? a.lay.OFF : 0))};
    {
        constexpr int kCla = fixed_cla(F);
        const int c1 = a.rm.c > 0 ? a.rm.c : 1;
        MH_CK(a.lay.CLA == kCla && a.lay.NZ == kCla + 16 * c1, 13, a.lay.CLA, kCla);
        ch.CLA = {reinterpret_cast<float4*>(base + kCla)};
        ch.NZ = {reinterpret_cast<uint64_t*>(base + kCla + 16 * c1)};
        ch.PRE = {reinterpret_cast<int*>(base + kCla + 32 * c1)};
    }
    ch.aux = {reinterpret_cast<ChainAux*>(base + F.AUX)};
    ch.rm = rm_l;
    ch.zero4 = reinterpret_cast<const double*>(lds + F.h_zero);

    // Zero the dense replay streams past N (never written afterwards).
    for (int i = n + r; i < a.lay.N4; i += L) {
        stage(ch.PX).put(i, 0.0);
        stage(ch.PY).put(i, 0.0);
        stage(ch.CPHF).put(i, 0.0);
        stage(ch.RMXF).put(i, 0.0);
    }
    // Stage the configuration: double poses into this lane's registers, float pose words
    // into LDS.
    const double* src;
    if constexpr (OP == OP_INIT) src = a.cfg;
    else if constexpr (OP == OP_EVAL) src = a.cfg + chain * (int64_t)(F_COUNT * n);
    else src = a.st + chain * (int64_t)(F_COUNT * n);
    OwnPose<NPL> op;
#pragma unroll
    for (int m = 0; m < NPL; ++m) {
        const int i = m * L + r;
        op.x[m] = op.y[m] = op.ry[m] = 0.0;
        if (i < n) {
            const double x = src[F_X * n + i], y = src[F_Y * n + i];
            const double ry = src[F_RY * n + i];
            op.x[m] = x;
            op.y[m] = y;
            op.ry[m] = ry;
            if constexpr (OP == OP_INIT) {  // z, rotX, rotZ live in HBM only
                ch.zrr[i] = src[F_Z * n + i];
                ch.zrr[n + i] = src[F_RX * n + i];
                ch.zrr[2 * n + i] = src[F_RZ * n + i];
            }
            ObjP p;
            p.xf = (float)x;
            p.yf = (float)y;
            p.rotYf = (float)ry;
            p.pad = 0.0f;
            stage(ch.P).put(i, p);
        }
    }
    // the staged configuration and the replay streams' zero tails
    hand_off(ch.P, ch.PX, ch.PY, ch.CPHF, ch.RMXF);

    float cur[8];
    SymRows<NPL> sym;  // symmetry row maxima of the current configuration
    if constexpr (OP == OP_INIT) {
        ClPairs cl0;
        eval_costs<L, NPL, false, false>(a, ch, op, r, gbase, cur, sym, sym, -1, -1, cl0, cl0);
        if (r == 0) {
            ChainMeta m;
            m.draws = 0;
            m.accepted = 0;
            m.bm_has = 0;
            m.bm_val = 0.0f;
            for (int k = 0; k < 8; ++k) m.costs[k] = cur[k];
            m.best_total = cur[0];  // cfgBest := the initial configuration, Kernel.cu:779-782
            m.rung = a.n_temps > 1 ? (int)((a.chain_offset + chain) % a.n_temps) : 0;
            a.meta[chain] = m;
        }
    } else if constexpr (STEP) {
        const ChainMeta m0 = a.meta[chain];
        const bool writer = (r == 0);
        if (writer)
            for (int k = 0; k < 8; ++k) stage(ch.aux)->cur[k] = m0.costs[k];
        float cur_total = m0.costs[0];
        bool cur_exact = true;  // (plain steps: false after a proposal accepted on the bound)
        CostIv cur_iv{cur_total, cur_total};
#if MH_CHECK
        float chk_cur = cur_total;  // (check builds: the current total, always exact)
#endif
        Rng rng;
        if constexpr (std::is_same<Rng, WaveRngLds>::value) {
            rng.bsl = reinterpret_cast<float*>(base + F.RNG);
            rng.ss = stage(ch.aux)->rng_key;  // (WaveRngLds hands its key words off itself)
        }
        rng_load(rng, a, chain, m0);
        // This launch's accepted count (at most `iterations`); the meta record's count, rung and
        // best total are re-read at the end rather than kept in scalar registers across the
        // steps (config 2 4.01 -> 3.93 ms per launch together with WaveRngLds's offset).
        unsigned int accepted = 0;
        float best_total = m0.best_total;
        double beta = kBeta;
        if constexpr (TRACK)  // (the extended families also carry parallel tempering)
            if (a.n_temps > 1) beta = a.ladder[m0.rung];
        ClPairs cl;  // non-zero Clearance pairs of the current configuration
        eval_costs<L, NPL, false, false>(a, ch, op, r, gbase, cur, sym, sym, -1, -1, cl, cl);
#if MH_STAMPS
        if (writer)
            for (int k = 0; k < 12; ++k) stage(ch.aux)->cyc[k] = 0;
        // the loop's shader cycles beside the constant 100 MHz counter: the clock it ran at
        unsigned long long loop_c0 = 0, loop_r0 = 0;
        MH_STAMP(loop_c0);
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(loop_r0) :: "memory");
#endif
#pragma clang loop unroll(disable)
        for (int it = 0; it < a.iterations; ++it) {
            unsigned long long ts = 0;
            MH_STAMP(ts);
            rng_prepare(rng);
            const int2 kk = propose<L, NPL>(rng, OP == OP_STEP_FEW ? a.rm : *rm_l, frozen, ch, op,
                                            r, gbase, writer);
            MH_CK(kk.x < n && kk.y < n && kk.x >= -1 && kk.y >= -1, 11, kk.x, kk.y);
            hand_off(ch.P, ch.aux);  // the proposal's pose words and its undo record
            if (writer) MH_PHASE(ch, 0, ts);
            float sc[8];
            SymRows<NPL> ss;
            ClPairs cls;
            // Steps of plain chains, one per wavefront: Accept's uniform (the next draw after the
            // proposal's, Kernel.cu:710) is drawn first, so a proposal the rejection bound
            // already rejects skips the exact sums (eval_costs FAST).
            // A proposal the bound accepts is taken without its exact costs: the current total is
            // then known as an interval (cur_iv) until a step needs it exactly (below).
            constexpr bool FASTK = !TRACK && FASTK_OF(L, NPL);
            int fast = BOUND_OPEN;
            CostIv star_iv{0.0f, 0.0f};
            float u_acc = 0.0f;
            if constexpr (FASTK) u_acc = rng.uniform();
            eval_costs<L, NPL, false, true, FASTK, OP == OP_STEP_FEW>(
                a, ch, op, r, gbase, sc, ss, sym, kk.x, kk.y, cls, cl, u_acc, cur_iv, &fast,
                &star_iv, true);
            // (exact costs only; a scalar register where the chain owns the wavefront)
            const float star0 = fast != BOUND_OPEN ? 0.0f : L == 64 ? uniform_f(sc[0]) : sc[0];
            MH_STAMP(ts);
#if MH_CHECK
            if constexpr (FASTK)
                if (r == 0) mh_count_decision(fast, true);
            // Check builds verify every decision the bound takes against the exact costs: the
            // proposal's exact total lies in the bound's interval, the current total in the
            // carried one, and a certain REJECT / ACCEPT is Accept's decision.
            float chk_star = star0;
            if constexpr (FASTK) {
                if (fast != BOUND_OPEN) {
                    float cx[8];
                    SymRows<NPL> sx;
                    ClPairs clx;
                    eval_costs<L, NPL, false, true>(a, ch, op, r, gbase, cx, sx, sym, kk.x, kk.y,
                                                    clx, cl);
                    chk_star = uniform_f(cx[0]);
                    if (r == 0) atomicAdd(&g_check[5], 1u);
                    const bool acc_x =
                        u_acc < accept_threshold(kBeta * ((double)chk_star - (double)chk_cur));
                    if (r == 0) {
                        MH_CK(chk_star >= star_iv.lo && chk_star <= star_iv.hi, 22,
                              __float_as_uint(chk_star), __float_as_uint(star_iv.hi - star_iv.lo));
                        MH_CK(fast != BOUND_REJECT || !acc_x, 20, __float_as_uint(chk_star),
                              __float_as_uint(chk_cur));
                        MH_CK(fast != BOUND_ACCEPT || acc_x, 21, __float_as_uint(chk_star),
                              __float_as_uint(chk_cur));
                    }
                }
                if (r == 0)
                    MH_CK(chk_cur >= cur_iv.lo && chk_cur <= cur_iv.hi, 23,
                          __float_as_uint(chk_cur), __float_as_uint(cur_iv.hi - cur_iv.lo));
            }
#endif
            if constexpr (FASTK) {
                // (rare: ~2% of config-3 steps; the hint lets the allocator keep the step's
                // values in registers around this path: 80 -> 72 bytes of scratch per lane,
                // 4.81e8 -> 4.84e8 chain-steps/s)
                // The proposal's exact total often decides against the current total's interval
                // alone (decide_exact_star); only otherwise is the current configuration made
                // exact.
                if (__builtin_expect(fast == BOUND_OPEN && !cur_exact, 0)) {
                    const int d2 = decide_exact_star(star0, cur_iv, u_acc, kBeta);
#if MH_CHECK
                    if (r == 0 && d2 != BOUND_OPEN) {
                        const bool acc_x = u_acc < accept_threshold(
                                               kBeta * ((double)star0 - (double)chk_cur));
                        MH_CK(acc_x == (d2 == BOUND_ACCEPT), 25, __float_as_uint(star0),
                              __float_as_uint(chk_cur));
                    }
#endif
                    if (d2 != BOUND_OPEN) fast = d2 + 32;  // (decided; the costs are exact)
                }
                if (__builtin_expect(fast == BOUND_OPEN && !cur_exact, 0)) {
                    // The decision needs the current configuration's exact costs: undo the
                    // proposal, evaluate the current configuration incrementally from the
                    // proposal's state (the same two objects differ), and keep the proposal's
                    // poses in the backup slots so that restore() re-applies them.
                    const int nb = ch.aux->nb;
                    const int k0 = nb > 0 ? ch.aux->b[0].k : 0, k1 = nb > 1 ? ch.aux->b[1].k : 0;
                    MH_CK(nb >= 0 && nb <= 2 && k0 >= 0 && k0 < n && k1 >= 0 && k1 < n, 10,
                          k0 | (nb << 16), k1);
                    const Backup s0 = read_obj<L, NPL>(op, k0, gbase);
                    const Backup s1 = read_obj<L, NPL>(op, k1, gbase);
                    restore<L, NPL>(ch, op, r, writer, kk);
                    hand_off(ch.P, ch.aux);  // the current configuration again
                    float cx[8];
                    SymRows<NPL> sx;
                    ClPairs clx;
                    eval_costs<L, NPL, false, true>(a, ch, op, r, gbase, cx, sx, ss, kk.x, kk.y, clx,
                                                    cls);
                    if (writer) {
                        const Staged<ChainAux> ax = stage(ch.aux);
                        for (int k = 0; k < 8; ++k) ax->cur[k] = cx[k];
                        if (nb > 0) ax->b[0] = s0;
                        if (nb > 1) ax->b[1] = s1;
                    }
#if MH_STAMPS
                    if (writer) stage(ch.aux)->cyc[11] += 1;
#endif
                    cur_total = uniform_f(cx[0]);
                    cur_exact = true;
                    cur_iv = CostIv{cur_total, cur_total};
#if MH_CHECK
                    if (r == 0) {
                        MH_CK(cur_total == chk_cur, 24, __float_as_uint(cur_total),
                              __float_as_uint(chk_cur));
                        atomicAdd(&g_decide[3], 1ull);
                    }
#endif
                    hand_off(ch.aux);  // its exact costs, and the proposal's poses as the undo record
                    if (u_acc < accept_threshold(kBeta * ((double)star0 - (double)cur_total))) {
                        restore<L, NPL>(ch, op, r, writer, kk);  // the proposal again
                        fast = BOUND_ACCEPT + 1;  // accepted with exact costs (below)
                    } else {
                        fast = BOUND_REJECT + 16;  // rejected, already undone
                    }
                    hand_off(ch.P);
                }
            }
            // Best-of-chain: star is judged before Accept, Kernel.cu:808-816.
            if constexpr (TRACK) {
                if (a.track != TRACK_OFF && best_improves(a.track, star0, best_total)) {
                    best_total = star0;
                    save_best_pose<L, NPL>(ch, op, a.best + chain * (int64_t)(F_COUNT * n), n, r);
                }
            }
            bool acc;
            bool exact = true;  // accepted with its exact costs
            if constexpr (TRACK) acc = accept_at(rng, star0, cur_total, beta);
            else if constexpr (FASTK) {
                if (fast == BOUND_OPEN)
                    acc = u_acc < accept_threshold(kBeta * ((double)star0 - (double)cur_total));
                else
                    acc = fast == BOUND_ACCEPT || fast == BOUND_ACCEPT + 1 ||
                          fast == BOUND_ACCEPT + 32;
                exact = fast != BOUND_ACCEPT;
            } else acc = accept(rng, star0, cur_total);
            if (acc) {
                sym = ss;
                cl = cls;
                ++accepted;
#if MH_CHECK
                if constexpr (FASTK) chk_cur = chk_star;
#endif
                if (exact) {
                    cur_total = star0;
                    if constexpr (FASTK) {
                        cur_exact = true;
                        cur_iv = CostIv{cur_total, cur_total};
                    }
                } else if constexpr (FASTK) {
                    cur_exact = false;
                    cur_iv = star_iv;
                }
                if (writer) {
                    if (exact)
                        for (int k = 0; k < 8; ++k) stage(ch.aux)->cur[k] = ch.aux->star[k];
                    commit_swap_zrr(ch, n);
                }
            } else if (fast != BOUND_REJECT + 16) {
                restore<L, NPL>(ch, op, r, writer, kk);
            }
            hand_off(ch.P, ch.aux);  // the step's configuration and current costs
            if (writer) MH_PHASE(ch, 7, ts);
        }
        if (!cur_exact) {
            // The exact costs of the final configuration: an incremental evaluation with no
            // object changed recomputes only the ordered sums.
            float cx[8];
            SymRows<NPL> sx;
            ClPairs clx;
            eval_costs<L, NPL, false, true>(a, ch, op, r, gbase, cx, sx, sym, -1, -1, clx, cl);
            if (writer)
                for (int k = 0; k < 8; ++k) stage(ch.aux)->cur[k] = cx[k];
            hand_off(ch.aux);
        }
#if MH_STAMPS
        if (writer)
            for (int k = 0; k < 12; ++k) atomicAdd(&g_phase_cycles[k], ch.aux->cyc[k]);
        {
            unsigned long long c1 = 0, r1 = 0;
            MH_STAMP(c1);
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r1) :: "memory");
            if (writer) {
                atomicAdd(&g_phase_cycles[12], c1 - loop_c0);
                atomicAdd(&g_phase_cycles[13], r1 - loop_r0);
            }
        }
#endif
#if MH_CHECK
        if (!TRACK && FASTK_OF(L, NPL) && r == 0)  // a launch ends with exact current costs
            MH_CK(ch.aux->cur[0] == chk_cur, 26, __float_as_uint(ch.aux->cur[0]),
                  __float_as_uint(chk_cur));
#endif
        if (writer) {
            ChainMeta m;
            const ChainMeta m1 = a.meta[chain];  // (re-read: m0 need not stay live)
            m.accepted = m1.accepted + accepted;
            m.draws = rng_draws(rng);
            m.bm_has = rng.bm_has;
            m.bm_val = rng.bm_val;
            rng_save(rng, a, chain);
            for (int k = 0; k < 8; ++k) m.costs[k] = ch.aux->cur[k];
            m.best_total = TRACK ? best_total : m1.best_total;
            m.rung = m1.rung;
            if (MH_CK(chain >= 0 && chain < a.n_chains, 12, (unsigned)chain, 0)) a.meta[chain] = m;
        }
    } else {  // OP_FINAL / OP_EVAL: full costs including OffLimits
        ClPairs clf;
        // (debug builds: the OffLimits boxes -- this pass's one array past the step layout -- lie
        // inside the chain's LDS slot, and the launch's LDS covers every chain of the workgroup)
        MH_CK(a.lay.OFF >= F.end && a.lay.OFF + 16 * n <= a.lay.stride, 16, a.lay.OFF, a.lay.stride);
        eval_costs<L, NPL, true, false>(a, ch, op, r, gbase, cur, sym, sym, -1, -1, clf, clf);
        // Output slot: in [0, n_chains) (tempering: a rung of the chain's own group)
        const int64_t oi = out_index(a, chain);
        const bool oi_ok = MH_CK(oi >= 0 && oi < a.n_chains && oi / a.n_temps == chain / a.n_temps,
                                 14, (unsigned)oi, (unsigned)chain);
        if (r == 0 && oi_ok) {
            resultCosts rc;
            rc.totalCosts = cur[0];
            rc.PairWiseCosts = cur[1];
            rc.VisualBalanceCosts = cur[2];
            rc.FocalPointCosts = cur[3];
            rc.SymmetryCosts = cur[4];
            rc.ClearanceCosts = cur[5];
            rc.OffLimitsCosts = cur[6];
            rc.SurfaceAreaCosts = cur[7];
            a.costs[oi] = rc;
        }
        if constexpr (OP == OP_FINAL) {
#pragma unroll
            for (int m = 0; m < NPL; ++m) {
                const int i = m * L + r;
                if (i >= n || !oi_ok) break;
                point p;
                p.x = (float)op.x[m];
                p.y = (float)op.y[m];
                p.z = (float)ch.zrr[i];
                p.rotX = (float)ch.zrr[n + i];
                p.rotY = (float)op.ry[m];
                p.rotZ = (float)ch.zrr[2 * n + i];
                a.pts[oi * (int64_t)n + i] = p;
            }
        }
    }

    if constexpr (OP == OP_INIT || STEP) {
        double* dst = a.st + chain * (int64_t)(F_COUNT * n);
#pragma unroll
        for (int m = 0; m < NPL; ++m) {
            const int i = m * L + r;
            if (i >= n) break;
            dst[F_X * n + i] = op.x[m];
            dst[F_Y * n + i] = op.y[m];
            dst[F_RY * n + i] = op.ry[m];
        }
    }
    if constexpr (OP == OP_INIT) {
        if (a.track != TRACK_OFF) {  // cfgBest := cfgCurrent, Kernel.cu:779-782
            if (r == 0) stage(ch.aux)->swap_a = -1;
            hand_off(ch.aux);
            save_best_pose<L, NPL>(ch, op, a.best + chain * (int64_t)(F_COUNT * n), n, r);
        }
    }
}

#ifndef MH_CHAIN_STEP_TU
// ---- summary reduction (for the multi-GPU best-cost all-gather) ---------------------------

__global__ void __launch_bounds__(1024) mh_summary_kernel(const resultCosts* costs,
                                                          const ChainMeta* meta, int64_t n,
                                                          int64_t chain_offset, mh_summary* out) {
    __shared__ double s_sum[1024];
    __shared__ float s_best[1024];
    __shared__ int64_t s_arg[1024];
    __shared__ int64_t s_acc[1024];
    double sum = 0.0;
    float best = -INFINITY;
    int64_t arg = -1, acc = 0;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const float t = costs[i].totalCosts;
        sum += (double)t;
        if (t > best || arg < 0) {
            best = t;
            arg = i;
        }
        acc += (int64_t)meta[i].accepted;
    }
    s_sum[threadIdx.x] = sum;
    s_best[threadIdx.x] = best;
    s_arg[threadIdx.x] = arg;
    s_acc[threadIdx.x] = acc;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            const int o = threadIdx.x + w;
            s_sum[threadIdx.x] += s_sum[o];
            s_acc[threadIdx.x] += s_acc[o];
            const bool take = s_arg[o] >= 0 &&
                              (s_arg[threadIdx.x] < 0 || s_best[o] > s_best[threadIdx.x] ||
                               (s_best[o] == s_best[threadIdx.x] && s_arg[o] < s_arg[threadIdx.x]));
            if (take) {
                s_best[threadIdx.x] = s_best[o];
                s_arg[threadIdx.x] = s_arg[o];
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        mh_summary s;
        s.sum_total = s_sum[0];
        s.best_total = s_best[0];
        s.pad = 0;
        s.best_chain = s_arg[0] < 0 ? -1 : s_arg[0] + chain_offset;
        s.n_chains = n;
        s.accepted = s_acc[0];
        *out = s;
    }
}

// ---- RNG diagnostic: the exact draws a chain sees --------------------------------------

__global__ void mh_rng_kernel(uint64_t seed, uint64_t subsequence, int n, unsigned int* u32,
                              float* uni, float* nrm) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    ChainRng r;
    r.bm_has = 0;
    r.bm_val = 0.f;
    r.init(seed, subsequence, 0);
    for (int i = 0; i < n; ++i) u32[i] = r.next();
    r.init(seed, subsequence, 0);
    for (int i = 0; i < n; ++i) uni[i] = r.uniform();
    r.init(seed, subsequence, 0);
    for (int i = 0; i < n; ++i) nrm[i] = r.normal();
}

// ---- numerics diagnostic: the shared transcendentals (mh_math.h) on the probe arguments ------

__global__ void __launch_bounds__(256) mh_math_kernel(int fn, uint64_t start, uint64_t count,
                                                     double* out) {
    const int w = mh_probe_width(fn);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < count; k += stride) {
        double r[2];
        if (fn == MH_PROBE_ACCEPT) {  // the device's decision is the screened one (accept_u)
            float u;
            double x;
            mh_arg_accept(start + k, &u, &x);
            r[0] = accept_u(u, x) ? 1.0 : 0.0;
        } else {
            mh_math_probe(fn, start + k, r);
        }
        out[k * w] = r[0];
        if (w == 2) out[k * w + 1] = r[1];
    }
}

// ---- cuRAND XORWOW seeding: curand_init(seed + id, id, 0) per chain (Kernel.cu:159) --------

// rocRAND's xorwow_engine implements the same recurrence and the same 2^67-draw subsequence
// jump (its precomputed jump matrices depend only on the recurrence); it differs from cuRAND in
// the seed-scrambling constants alone. This engine applies cuRAND's constants
// (_curand_init_scratch in curand_kernel.h) and then rocRAND's subsequence jump.
struct CurandXorwowSeeder : rocrand_device::xorwow_engine {
    __device__ CurandXorwowSeeder(unsigned long long seed, unsigned long long subsequence)
        : rocrand_device::xorwow_engine(0ull, 0ull, 0ull) {
        const unsigned int s0 = (unsigned int)seed ^ 0xaad26b49u;
        const unsigned int s1 = (unsigned int)(seed >> 32) ^ 0xf7dcefddu;
        const unsigned int t0 = 1099087573u * s0;
        const unsigned int t1 = 2591861531u * s1;
        m_state.d = 6615241u + t1 + t0;
        m_state.x[0] = 123456789u + t0;
        m_state.x[1] = 362436069u ^ t0;
        m_state.x[2] = 521288629u + t1;
        m_state.x[3] = 88675123u ^ t1;
        m_state.x[4] = 5783321u + t0;
        discard_subsequence(subsequence);
    }
    __device__ void store(unsigned int* w) const {
        w[0] = m_state.d;
        for (int k = 0; k < 5; ++k) w[1 + k] = m_state.x[k];
    }
};

// Chain c (global id g = chain_offset + c) gets curand_init((unsigned)(seed + g), g, 0): the
// reference adds the thread id to an unsigned int seed (Kernel.cu:151-159,943).
__global__ void __launch_bounds__(256) mh_xorwow_init_kernel(uint64_t seed, int64_t chain_offset,
                                                             int64_t n, unsigned int* xw) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const uint64_t g = (uint64_t)(chain_offset + c);
    const CurandXorwowSeeder e((unsigned int)(seed + g), g);
    e.store(xw + c * 6);
}

__global__ void mh_rng_xw_kernel(uint64_t seed, uint64_t subsequence, int n, unsigned int* u32,
                                 float* uni, float* nrm) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    unsigned int w[6];
    CurandXorwowSeeder(seed, subsequence).store(w);
    ChainRngXw r;
    for (int pass = 0; pass < 3; ++pass) {
        r.d = w[0];
        r.x0 = w[1];
        r.x1 = w[2];
        r.x2 = w[3];
        r.x3 = w[4];
        r.x4 = w[5];
        r.draws = 0;
        r.bm_has = 0;
        r.bm_val = 0.f;
        for (int i = 0; i < n; ++i) {
            if (pass == 0) u32[i] = r.next();
            else if (pass == 1) uni[i] = r.uniform();
            else nrm[i] = r.normal();
        }
    }
}

// ---- parallel tempering: one replica-exchange round ----------------------------------------

// One thread per group of K = n_temps chains. perm[g*K + k] is the group-local index of the
// chain at rung k. Round t tries the disjoint rung pairs (k, k+1), k = (t-1) mod 2 + 2i, with
// the Philox uniform (key = seed, subsequence = 2^63 + global group, offset = (t-1)*K + k) and
// the exchange rule for pi_beta ~ exp(beta * totalCosts) (the maximisation Accept performs).
__global__ void __launch_bounds__(256) mh_exchange_kernel(LaunchArgs a, int* perm, int round) {
    const int K = a.n_temps;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g * K >= a.n_chains) return;
    int* pg = perm + g * K;
    ChainMeta* mg = a.meta + g * K;
    const uint64_t gid = (uint64_t)(a.chain_offset / K + g);
    for (int k = (round - 1) & 1; k + 1 < K; k += 2) {
        const int ca = pg[k], cb = pg[k + 1];
        const float ea = mg[ca].costs[0], eb = mg[cb].costs[0];
        rocrand_state_philox4x32_10 st;
        rocrand_init(a.seed, (1ull << 63) | gid, (uint64_t)(round - 1) * K + k, &st);
        const float u = rocrand_device::detail::uniform_distribution(rocrand(&st));
        const double db = a.ladder[k] - a.ladder[k + 1];
        const float thr = fminf(1.0f, (float)mh_exp(db * ((double)eb - (double)ea)));
        if (u < thr) {
            pg[k] = cb;
            pg[k + 1] = ca;
            mg[ca].rung = k + 1;
            mg[cb].rung = k;
        }
    }
}

// ---- diagnostic: the group collectives on given lane values ---------------------------------

// out[k * 64 + lane] for k = 0 top-2 m1, 1 m2, 2 argmax (lane index within the group, values
// v), 3 max-with-index value, 4 its index, 5 exclusive scan of iv, 6 its group total,
// 7 group max of iv, 8 group sum of iv (floats as bits), 9..16 the eight wavefront sums of
// wave_fsum8 over the lane values (float)(iv[(3 lane + k) & 63] + k), k = 0..7 (floats as bits).
template <int L>
__global__ void mh_collectives_kernel(const float* v, const int* iv, int* out) {
    const int lane = threadIdx.x;
    const int r = lane % L;
    float m1 = v[lane], m2 = -INFINITY;
    int j1 = r;
    group_top2<L>(m1, m2, j1);
    float mv = v[lane];
    int mj = r;
    group_max_arg<L>(mv, mj);
    int tot;
    const int ex = group_excl_scan<L>(iv[lane], r, tot);
    out[0 * 64 + lane] = __float_as_int(m1);
    out[1 * 64 + lane] = __float_as_int(m2);
    out[2 * 64 + lane] = j1;
    out[3 * 64 + lane] = __float_as_int(mv);
    out[4 * 64 + lane] = mj;
    out[5 * 64 + lane] = ex;
    out[6 * 64 + lane] = tot;
    out[7 * 64 + lane] = group_max<L>(iv[lane]);
    out[8 * 64 + lane] = group_sum<L>(iv[lane]);
    float part[8], sum[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) part[k] = (float)(iv[(3 * lane + k) & 63] + k);
    wave_fsum8(part, sum);
#pragma unroll
    for (int k = 0; k < 8; ++k) out[(9 + k) * 64 + lane] = __float_as_int(sum[k]);
}

// ---- host-side launch dispatch ------------------------------------------------------------

template <int L, int NPL>
static hipError_t launch_geom(int op, const LaunchArgs& a, int waves_per_wg, hipStream_t stream) {
    constexpr int G = 64 / L;
    const int64_t chains_per_wg = (int64_t)waves_per_wg * G;
    const int64_t blocks = (a.n_chains + chains_per_wg - 1) / chains_per_wg;
    const size_t lds = (size_t)a.lay.hdr + (size_t)waves_per_wg * G * a.lay.stride;
    const dim3 grid((unsigned)blocks), block((unsigned)(64 * waves_per_wg));
    switch (op) {
        case OP_INIT: hipLaunchKernelGGL((mh_kernel<L, NPL, OP_INIT>), grid, block, lds, stream, a); break;
        case OP_STEP: hipLaunchKernelGGL((mh_kernel<L, NPL, OP_STEP>), grid, block, lds, stream, a); break;
        case OP_STEP_FEW:
            if constexpr (L == 64 && NPL == 1)
                hipLaunchKernelGGL((mh_kernel<64, 1, OP_STEP_FEW>), grid, block, lds, stream, a);
            else
                hipLaunchKernelGGL((mh_kernel<L, NPL, OP_STEP>), grid, block, lds, stream, a);
            break;
        case OP_FINAL: hipLaunchKernelGGL((mh_kernel<L, NPL, OP_FINAL>), grid, block, lds, stream, a); break;
        default: hipLaunchKernelGGL((mh_kernel<L, NPL, OP_EVAL>), grid, block, lds, stream, a); break;
    }
    return hipGetLastError();
}

}  // namespace mh

// Entry points used by mh_abi.cpp.
namespace mh {

// Lanes per chain: the next power of two >= N (at least 8, at most 64); objects per lane
// (NPL) covers N > 64. When the chains are too few to fill the GPU at that width, chains get
// wider, up to a wavefront each, while their waves still fit `resident_waves` (a step's
// critical path is shorter with one chain per wavefront: readlane instead of ds_bpermute, the
// wave-batched RNG, the incremental clearance and atan2 passes; config 2, N = 8 x 1,024 chains:
// 9.0e7 chain-steps/s at L = 8, 1.24e8 at 32, 1.73e8 at 64). $MH_LANES pins the width.
int choose_lanes(int n, int64_t n_chains, int64_t resident_waves) {
    int L = 8;
    while (L < n && L < 64) L <<= 1;
    if (const char* e = getenv("MH_LANES")) {  // tuning override: 8, 16, 32 or 64
        const int want = atoi(e);
        if ((want == 8 || want == 16 || want == 32 || want == 64) && (n + want - 1) / want <= 8)
            return want;
    }
    while (L < 64 && n_chains * (2 * L) <= resident_waves * 64) L <<= 1;
    return L;
}
int choose_npl(int n, int L) { return (n + L - 1) / L; }
int max_npl() { return 8; }

// Resident workgroups per CU of the plain step kernel for a launch shape (registers, LDS and
// the wave limit, as the runtime counts them). 0 if it does not fit.
template <int L>
static int step_blocks_l(int npl, int threads, size_t lds, bool few) {
    int blocks = 0;
    hipError_t e;
    if (few && L == 64 && npl <= 1)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_kernel<64, 1, OP_STEP_FEW>, threads, lds);
    else if (npl <= 1) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_kernel<L, 1, OP_STEP>, threads, lds);
    else if (npl <= 2) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_kernel<L, 2, OP_STEP>, threads, lds);
    else if (npl <= 4) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_kernel<L, 4, OP_STEP>, threads, lds);
    else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_kernel<L, 8, OP_STEP>, threads, lds);
    return e == hipSuccess ? blocks : 0;
}

int step_blocks_per_cu(int L, int npl, int waves_per_wg, size_t lds, bool few) {
    const int threads = 64 * waves_per_wg;
    switch (L) {
        case 8: return step_blocks_l<8>(npl, threads, lds, false);
        case 16: return step_blocks_l<16>(npl, threads, lds, false);
        case 32: return step_blocks_l<32>(npl, threads, lds, false);
        default: return step_blocks_l<64>(npl, threads, lds, few);
    }
}

size_t lds_bytes(const ChainLds& lay, int L, int waves_per_wg) {
    return (size_t)lay.hdr + (size_t)waves_per_wg * (64 / L) * lay.stride;
}

hipError_t launch(int op, const LaunchArgs& a, int L, int npl, int waves_per_wg, hipStream_t s) {
    if (a.n_chains <= 0) return hipSuccess;
    const bool step = op == OP_STEP || op == OP_STEP_FEW;
    if (step && a.rng == RNG_CURAND_XORWOW) return launch_step_xw(a, L, npl, waves_per_wg, s);
    if (step && (a.track != TRACK_OFF || a.n_temps > 1))
        return launch_step_best(a, L, npl, waves_per_wg, s);
    // (lanes per chain, objects per lane) instantiations; npl rounds up to the next one.
    switch (L) {
        case 8:
            if (npl <= 1) return launch_geom<8, 1>(op, a, waves_per_wg, s);
            if (npl <= 2) return launch_geom<8, 2>(op, a, waves_per_wg, s);
            if (npl <= 4) return launch_geom<8, 4>(op, a, waves_per_wg, s);
            return launch_geom<8, 8>(op, a, waves_per_wg, s);
        case 16:
            if (npl <= 1) return launch_geom<16, 1>(op, a, waves_per_wg, s);
            if (npl <= 2) return launch_geom<16, 2>(op, a, waves_per_wg, s);
            if (npl <= 4) return launch_geom<16, 4>(op, a, waves_per_wg, s);
            return launch_geom<16, 8>(op, a, waves_per_wg, s);
        case 32:
            if (npl <= 1) return launch_geom<32, 1>(op, a, waves_per_wg, s);
            if (npl <= 2) return launch_geom<32, 2>(op, a, waves_per_wg, s);
            if (npl <= 4) return launch_geom<32, 4>(op, a, waves_per_wg, s);
            return launch_geom<32, 8>(op, a, waves_per_wg, s);
        default:
            if (npl <= 1) return launch_geom<64, 1>(op, a, waves_per_wg, s);
            if (npl <= 2) return launch_geom<64, 2>(op, a, waves_per_wg, s);
            if (npl <= 4) return launch_geom<64, 4>(op, a, waves_per_wg, s);
            return launch_geom<64, 8>(op, a, waves_per_wg, s);
    }
}

hipError_t launch_summary(const resultCosts* costs, const ChainMeta* meta, int64_t n,
                          int64_t chain_offset, mh_summary* out, hipStream_t s) {
    hipLaunchKernelGGL(mh_summary_kernel, dim3(1), dim3(1024), 0, s, costs, meta, n, chain_offset, out);
    return hipGetLastError();
}

#if MH_CHECK
extern "C" __attribute__((visibility("default"))) int mh_debug_check(unsigned int* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_check), sizeof(unsigned int) * 8) == hipSuccess ? 0 : -1;
}
extern "C" __attribute__((visibility("default"))) int mh_debug_decisions(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_decide), sizeof(unsigned long long) * 4) ==
                   hipSuccess ? 0 : -1;
}
#endif

#if MH_STAMPS
extern "C" __attribute__((visibility("default"))) int mh_debug_phase_cycles(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_cycles), sizeof(unsigned long long) * 14) ==
                   hipSuccess ? 0 : -1;
}
#endif

hipError_t launch_collectives(int L, const float* v, const int* iv, int* out, hipStream_t s) {
    switch (L) {
        case 8: hipLaunchKernelGGL(mh_collectives_kernel<8>, dim3(1), dim3(64), 0, s, v, iv, out); break;
        case 16: hipLaunchKernelGGL(mh_collectives_kernel<16>, dim3(1), dim3(64), 0, s, v, iv, out); break;
        case 32: hipLaunchKernelGGL(mh_collectives_kernel<32>, dim3(1), dim3(64), 0, s, v, iv, out); break;
        default: hipLaunchKernelGGL(mh_collectives_kernel<64>, dim3(1), dim3(64), 0, s, v, iv, out); break;
    }
    return hipGetLastError();
}

hipError_t launch_rng(int kind, uint64_t seed, uint64_t subsequence, int n, unsigned int* u32,
                      float* uni, float* nrm, hipStream_t s) {
    if (kind == RNG_CURAND_XORWOW)
        hipLaunchKernelGGL(mh_rng_xw_kernel, dim3(1), dim3(64), 0, s, seed, subsequence, n, u32, uni, nrm);
    else
        hipLaunchKernelGGL(mh_rng_kernel, dim3(1), dim3(64), 0, s, seed, subsequence, n, u32, uni, nrm);
    return hipGetLastError();
}

hipError_t launch_math(int fn, uint64_t start, uint64_t count, double* out, hipStream_t s) {
    if (count == 0) return hipSuccess;
    const uint64_t blocks = (count + 255) / 256 < 65536 ? (count + 255) / 256 : 65536;
    hipLaunchKernelGGL(mh_math_kernel, dim3((unsigned)blocks), dim3(256), 0, s, fn, start, count, out);
    return hipGetLastError();
}

hipError_t launch_exchange(const LaunchArgs& a, int* perm, int round, hipStream_t s) {
    const int64_t groups = a.n_chains / a.n_temps;
    if (groups <= 0) return hipSuccess;
    hipLaunchKernelGGL(mh_exchange_kernel, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, s,
                       a, perm, round);
    return hipGetLastError();
}

hipError_t launch_xorwow_init(uint64_t seed, int64_t chain_offset, int64_t n, unsigned int* xw,
                              hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(mh_xorwow_init_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       seed, chain_offset, n, xw);
    return hipGetLastError();
}

}  // namespace mh
#else  // MH_CHAIN_STEP_TU: one more family of step kernels (mh_chain_xw.hip, mh_chain_best.hip)

template <int L, int NPL>
static hipError_t launch_geom_step(const LaunchArgs& a, int waves_per_wg, hipStream_t stream) {
    constexpr int G = 64 / L;
    const int64_t chains_per_wg = (int64_t)waves_per_wg * G;
    const int64_t blocks = (a.n_chains + chains_per_wg - 1) / chains_per_wg;
    const size_t lds = (size_t)a.lay.hdr + (size_t)waves_per_wg * G * a.lay.stride;
    hipLaunchKernelGGL((mh_kernel<L, NPL, MH_CHAIN_STEP_TU>), dim3((unsigned)blocks),
                       dim3((unsigned)(64 * waves_per_wg)), lds, stream, a);
    return hipGetLastError();
}

hipError_t MH_CHAIN_STEP_LAUNCH(const LaunchArgs& a, int L, int npl, int waves_per_wg, hipStream_t s) {
    switch (L) {
        case 8:
            if (npl <= 1) return launch_geom_step<8, 1>(a, waves_per_wg, s);
            if (npl <= 2) return launch_geom_step<8, 2>(a, waves_per_wg, s);
            if (npl <= 4) return launch_geom_step<8, 4>(a, waves_per_wg, s);
            return launch_geom_step<8, 8>(a, waves_per_wg, s);
        case 16:
            if (npl <= 1) return launch_geom_step<16, 1>(a, waves_per_wg, s);
            if (npl <= 2) return launch_geom_step<16, 2>(a, waves_per_wg, s);
            if (npl <= 4) return launch_geom_step<16, 4>(a, waves_per_wg, s);
            return launch_geom_step<16, 8>(a, waves_per_wg, s);
        case 32:
            if (npl <= 1) return launch_geom_step<32, 1>(a, waves_per_wg, s);
            if (npl <= 2) return launch_geom_step<32, 2>(a, waves_per_wg, s);
            if (npl <= 4) return launch_geom_step<32, 4>(a, waves_per_wg, s);
            return launch_geom_step<32, 8>(a, waves_per_wg, s);
        default:
            if (npl <= 1) return launch_geom_step<64, 1>(a, waves_per_wg, s);
            if (npl <= 2) return launch_geom_step<64, 2>(a, waves_per_wg, s);
            if (npl <= 4) return launch_geom_step<64, 4>(a, waves_per_wg, s);
            return launch_geom_step<64, 8>(a, waves_per_wg, s);
    }
}

}  // namespace mh
#endif  // MH_CHAIN_STEP_TU
