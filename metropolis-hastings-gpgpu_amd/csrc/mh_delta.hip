// mh_delta.hip -- the MH step (Kernel.cu:785-828) with incremental cost evaluation.
//
// A proposal changes at most two objects (propose(), Kernel.cu:576-704), so almost every term
// of Costs() (Kernel.cu:516-550) is the same before and after it. This kernel keeps, per chain,
// every quantity a proposal can only change locally, recomputes just the affected entries, and
// replays the reference's ordered float/double sums from the cached terms:
//   * FocalPoint: -cos(phi_i) per object (an LDS stream, the replay reads it as it lies);
//   * Symmetry: each row's exact maximum and its argmax, in the row owner's registers (current
//     and proposed); a proposal re-scans the changed rows and folds the changed columns into
//     the others;
//   * Clearance: the non-zero (clearance, object) overlap pairs as a bit matrix, updated by
//     row (clearances whose source moved) and by column (moved objects);
//   * SurfaceArea: a bit per non-zero entry;
//   * PairWise / PairWiseAngle: the term of every relationship, recomputed when one of its
//     objects moved;
//   * VisualBalance needs no cache (area * x is one product).
// The values that enter every sum are the reference's own (same functions as the full
// evaluation, mh_common.h); only the work to find them changes, so costs -- and chains -- stay
// bit-identical to the oracle.
//
// One chain owns one 64-lane wavefront; lane r owns objects r + 64 s (s < S slots, S =
// ceil(N / 64)). The kernel is latency-bound (a step is a chain of short dependent passes), so
// its throughput is the number of chains a CU keeps resident, and that is set by LDS per chain:
// whatever only the owner lane reads (rotY, the symmetry rows) lives in registers, and LDS holds
// what other lanes read (poses, object and clearance boxes, pair bits) and the replay streams.

#include <stdint.h>
#include <stdlib.h>

#ifndef MH_MATH_OOL
#define MH_MATH_OOL 1  // atan2 out of line in the incremental kernel (config 5: 1% faster)
#endif
#include "mh_common.h"

#ifndef MH_STAMPS
#define MH_STAMPS 0  // diagnostic builds: cycles per phase of the step (tools/stamps.py)
#endif
#if MH_STAMPS
__device__ unsigned long long g_delta_cycles[8];
// sums of the Clearance / SurfaceArea list sizes, list overflows, steps that evaluated the
// rejection bound, steps it rejected, steps it accepted, exact passes of the current configuration
__device__ unsigned long long g_delta_counts[8];
#define DSTAMP(k) do { __builtin_amdgcn_sched_barrier(0); unsigned long long _t; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t) :: "memory"); cyc[k] += _t - t_last; t_last = _t; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define DSTAMP(k) do { } while (0)
#endif

namespace mh {
namespace {

constexpr int L = 64;  // lanes per chain: one chain per wavefront

struct RowMax {  // one symmetry row: exact max(0, max_j value) and the j attaining it (-1: 0)
    float mx;
    int arg;
};

// Registers of one chain, per owner lane: the pose of objects r + 64 s and the symmetry rows
// (current configuration; proposed configuration). Vector types, so that no access -- not even
// one whose slot differs between lanes -- sends them to scratch: an array of S elements indexed
// by a select chain was folded into an indexed load of a stack slot.
template <int S>
struct Own {
    typedef double dvec __attribute__((ext_vector_type(S)));
    typedef float fvec __attribute__((ext_vector_type(S)));
    typedef int ivec __attribute__((ext_vector_type(S)));
    typedef unsigned long long wvec __attribute__((ext_vector_type(S)));
    dvec ry;
    fvec xf, yf;  // (float)x, (float)y
    fvec cmx;
    ivec carg;
    fvec pmx;
    ivec parg;
    wvec nz0;  // the non-zero Clearance pair words of clearance r (rows >= 64 live in LDS)
    float4 cla0;  // clearance r's box at its source object (clearances >= 64: LDS)
    // SurfaceArea entry e = 64 t + r (t < 2S: C + N <= 128 S) of the current configuration, as
    // the rejection bound sums it: (v.x + v.y) + (v.z + v.w) of its four overlaps (zero when
    // they all are), so a step the bound decides builds no SurfaceArea list
    typedef float svec __attribute__((ext_vector_type(2 * S)));
    svec sav;
};

// v[m] = x where pred holds (m may differ between lanes).
template <int S, typename V, typename T>
__device__ __forceinline__ void slot_put(V& v, int m, T x, bool pred) {
#pragma unroll
    for (int q = 0; q < S; ++q) v[q] = (pred && q == m) ? x : v[q];
}

// rotY of object k (wave-uniform k), from its owner lane.
template <int S>
__device__ __forceinline__ double obj_ry(const Own<S>& o, int k) {
    return grp_get<L>((double)o.ry[k >> 6], k & 63, 0);
}

struct DBackup {  // an object's cost-relevant pose and FocalPoint term before a proposal
    int k;
    float w;
    double x, y, ry;
};

struct DeltaAux {  // (the current configuration's resultCosts live in registers)
    DBackup b[2];
    int nb;
    int swap_a, swap_b;
    int pad0;
};
static_assert(sizeof(DeltaAux) <= kDeltaAuxBytes, "DeltaAux");

struct DeltaPtrs {
    const RectShape* objs;  // object off-limits rectangles
    const RectShape* clrs;  // clearance rectangles, the source object in .pad
    const uint2* rel;       // LDS: relationship objects {s | t << 16, as | at << 16} (hit test)
    const RelConst* relg;   // HBM: the relationship records (read for the ones a move touches)
    const float4* rele;     // HBM: their fp32 estimate constants, e0[nre] then e1[nre]
    int nre;                // max(R, 1)
    const DevRoom* rm;
    const float *AREA, *ONES;  // replay streams shared by the workgroup
    const double* ZERO;   // double[DL] zeros
    const float* ZEROF;   // 4 zero floats
    // (every array that one lane writes and other lanes read is a Published view, mh_common.h:
    // lanes write through stage(ch.X), and each phase ends in hand_off(ch.X, ...))
    Published<double> X, Y;
    Published<float4> BOX;  // object off-limits boxes at the current poses, zero past N
    Published<float> RYF;   // (float)rotY
    Published<float> CPH;   // -cos(phi): the FocalPoint terms (the replay's stream), zero past N
    Published<float> NMX;   // -(row max) of the proposed rows: the replay's Symmetry stream
    Published<float4> CLA;  // boxes of clearances 64.. (the first 64: registers, Own::cla0)
    Published<uint64_t> NZ;  // pair words of clearances 64.. (the first 64 rows: registers, Own::nz0)
    Published<uint32_t> SAM, SAMB;
    Published<double> RPW, RANG;
    Published<float> LCL, LSA;
    Published<DeltaAux> aux;  // (the writer lane's record)
    double* zrr;  // HBM: z, rotX, rotZ rows of this chain
    int W, SW, cap_cl, cap_sa, NP, NR, DL;
};

// ---- per-object quantities --------------------------------------------------------------------

__device__ __forceinline__ float4 obj_box(const DeltaPtrs& ch, int j) { return ch.BOX[j]; }

// Object k's float pose {xf, yf, rotYf} (the .pad word is not set).
__device__ __forceinline__ ObjP obj_pose(const DeltaPtrs& ch, int k) {
    ObjP p;
    p.xf = (float)ch.X[k];
    p.yf = (float)ch.Y[k];
    p.rotYf = ch.RYF[k];
    p.pad = 0.0f;
    return p;
}

__device__ __forceinline__ float4 cla_box(const DeltaPtrs& ch, int ci) {
    const RectShape& cs = ch.clrs[ci];
    return shape_box(cs, (float)ch.X[cs.pad], (float)ch.Y[cs.pad]);
}

// Clearance ci's box: its owner lane's register (ci < 64) or LDS. `own`: this lane owns ci.
template <int S>
__device__ __forceinline__ float4 cla_get(const DeltaPtrs& ch, const Own<S>& o, int ci) {
    if (ci < 64) return o.cla0;  // (not a ?: of the two lvalues: a select of their addresses
    return ch.CLA[ci - 64];      // put the register copy in scratch)
}
template <int S>
__device__ __forceinline__ void cla_put(const DeltaPtrs& ch, Own<S>& o, int ci, float4 v) {
    if (ci < 64) o.cla0 = v;
    else stage(ch.CLA).put(ci - 64, v);
}

// SurfaceAreaCosts entry e (Kernel.cu:453-480): clearance e's box at cfg[e] (the reference's
// quirk, :456) for e < C, then object e - C's off-limits box.
__device__ __forceinline__ float4 sa_entry(const DeltaPtrs& ch, int c, int e) {
    if (e < c)
        return comp_overlaps(*ch.rm, shape_box(ch.clrs[e], (float)ch.X[e], (float)ch.Y[e]));
    return comp_overlaps(*ch.rm, obj_box(ch, e - c));
}

// FocalPointCosts term of object i, Kernel.cu:271,277 with phi() of :185-188.
__device__ __forceinline__ float focal_cos(const DevRoom& rm, float xf, float yf, float ryf) {
    const float at = atan2_f32(rm.fyf - yf, rm.fxf - xf);
    const float b = at - ryf;
    const float ph = (float)((double)b + kHalfPI);
    return cos_f32(ph);
}

// SymmetryCosts row setup of object i (rotY ryi), Kernel.cu:292-299.
__device__ __forceinline__ void row_setup(const DeltaPtrs& ch, int i, double ryi, float& rx,
                                          float& ry, float& rr) {
    const DevRoom& rm = *ch.rm;
    const double x = ch.X[i], y = ch.Y[i];
    double al = x * (double)rm.ux;
    al = al + y * (double)rm.uy;
    const float sd = (float)(2.0 * (rm.along_f - al));
    rx = (float)(x + (double)(sd * rm.ux));
    ry = (float)(y + (double)(sd * rm.uy));
    float t = (float)(rm.two_focal_rot - ryi);
    if ((double)t < -kPI) t = (float)((double)t + kTwoPI);
    rr = t;
}

__device__ __forceinline__ bool wild_pose(double x, double y, double ry) {
    return !(fabs(x) < 1e15 && fabs(y) < 1e15 && fabs(ry) < 1e15);
}

__device__ __forceinline__ void sam_put(const DeltaPtrs& ch, int e, bool nz) {
    const uint32_t bit = 1u << (e & 31);
    if (nz) atomicOr(stage(ch.SAM).ptr() + (e >> 5), bit);
    else atomicAnd(stage(ch.SAM).ptr() + (e >> 5), ~bit);
}

// ---- symmetry rows ------------------------------------------------------------------------

// Exact row maximum of row i (wave-uniform) over every column, the lanes sharing the columns:
// fp32 estimates screen the pairs (sym_err bounds their error), the leader is evaluated exactly
// and an ambiguous top two falls back to the exact value of every candidate within the bound.
template <int S>
__device__ __forceinline__ RowMax scan_row(const DeltaPtrs& ch, const Own<S>& o, int n, int i, bool exact_mode,
                           int r) {
    float rx, ry, rr;
    row_setup(ch, i, obj_ry<S>(o, i), rx, ry, rr);
    float t1 = -INFINITY, t2 = -INFINITY;
    int tj = -1;
#pragma unroll
    for (int q = 0; q < S; ++q) {
        const int j = q * L + r;
        if (j < n) {
            const float v = sym_val_fast(make_float4(o.xf[q], o.yf[q], (float)o.ry[q], 0.0f), rx,
                                         ry, rr);
            t2 = __builtin_amdgcn_fmed3f(t1, t2, v);
            const bool up = v > t1;
            t1 = up ? v : t1;
            tj = up ? j : tj;
        }
    }
    const SymLead ld = group_sym_lead<L>(t1, t2, tj, r, 0, rr);
    RowMax out;
    if (!exact_mode && ld.clear) {
        const float e = sym_val_exact((float)ch.X[ld.j], (float)ch.Y[ld.j], obj_ry<S>(o, ld.j),
                                      rx, ry, (double)rr);
        out.mx = fmaxf(0.0f, e);
        out.arg = e > 0.0f ? ld.j : -1;
        return out;
    }
    const float thr =
        (exact_mode || ld.j < 0) ? INFINITY : 2.0f * sym_err(fabsf(ld.m) + 1.0f, rr);
    float bv = -INFINITY;
    int bj = -1;
#pragma unroll
    for (int q = 0; q < S; ++q) {
        const int j = q * L + r;
        if (j < n) {
            const float v = sym_val_fast(make_float4(o.xf[q], o.yf[q], (float)o.ry[q], 0.0f), rx,
                                         ry, rr);
            if (!(v < ld.m - thr)) {
                const float e = sym_val_exact(o.xf[q], o.yf[q], o.ry[q], rx, ry, (double)rr);
                if (e > bv) {
                    bv = e;
                    bj = j;
                }
            }
        }
    }
    group_max_arg<L>(bv, bj);
    out.mx = bv > 0.0f ? bv : 0.0f;
    out.arg = bv > 0.0f ? bj : -1;
    return out;
}

// Proposed rows (o.pmx / o.parg) of the configuration after objects ka, kb (-1: none) changed,
// from the current rows (o.cmx / o.carg). Lane r owns rows r + 64 s.
template <int S>
__device__ __forceinline__ void symmetry_delta(const DeltaPtrs& ch, Own<S>& o, int n, int ka, int kb,
                               bool exact_mode, int r) {
    float4 qa = make_float4(0.f, 0.f, 0.f, 0.f), qb = qa;
    if (ka >= 0) qa = make_float4((float)ch.X[ka], (float)ch.Y[ka], ch.RYF[ka], 0.0f);
    if (kb >= 0) qb = make_float4((float)ch.X[kb], (float)ch.Y[kb], ch.RYF[kb], 0.0f);
    const double rya = obj_ry<S>(o, ka < 0 ? 0 : ka), ryb = obj_ry<S>(o, kb < 0 ? 0 : kb);
    unsigned pa = 0, pb = 0, resc = 0;
#pragma unroll
    for (int t = 0; t < S; ++t) {
        const int i = t * L + r;
        o.pmx[t] = o.cmx[t];
        o.parg[t] = o.carg[t];
        if (i >= n) continue;
        if (i == ka || i == kb) {
            resc |= 1u << t;
            continue;
        }
        float rx, ry, rr;
        row_setup(ch, i, o.ry[t], rx, ry, rr);
        const float cm = o.cmx[t];
        const int ca = o.carg[t];
        // pending unless certainly below the old maximum; a maximum held by the changed
        // column that certainly dropped sends the row straight to the re-scan
        if (ka >= 0) {
            const float v = sym_val_fast(qa, rx, ry, rr);
            const bool below = !exact_mode && v + sym_err(v, rr) < cm;
            if (ca == ka && below) resc |= 1u << t;
            else if (!below) pa |= 1u << t;
        }
        if (kb >= 0) {
            const float v = sym_val_fast(qb, rx, ry, rr);
            const bool below = !exact_mode && v + sym_err(v, rr) < cm;
            if (ca == kb && below) resc |= 1u << t;
            else if (!below) pb |= 1u << t;
        }
    }
    pa &= ~resc;
    pb &= ~resc;
    // Exact values of the pending (row, column) pairs, one per lane per pass.
    while (__ballot((pa | pb) != 0)) {
        if (pa | pb) {
            int tt, col;
            double ryc;
            if (pa) {
                tt = __builtin_ctz(pa);
                pa &= pa - 1;
                col = ka;
                ryc = rya;
            } else {
                tt = __builtin_ctz(pb);
                pb &= pb - 1;
                col = kb;
                ryc = ryb;
            }
            const int i = tt * L + r;
            float rx, ry, rr;
            row_setup(ch, i, o.ry[tt], rx, ry, rr);
            const float4 q = col == ka ? qa : qb;
            const float e = sym_val_exact(q.x, q.y, ryc, rx, ry, (double)rr);
            const float cm = o.cmx[tt];
            const int ca = o.carg[tt];
            const float sm = o.pmx[tt];
            if (col == ca && !(e >= cm)) {
                resc |= 1u << tt;  // the old maximum is gone: re-scan the row
            } else if (e > sm) {
                slot_put<S>(o.pmx, tt, e, true);
                slot_put<S>(o.parg, tt, col, true);
            }
        }
    }
    // Re-scans, one row at a time across the chain's lanes.
    for (;;) {
        const uint64_t who = __ballot(resc != 0);
        if (who == 0) break;
        const int b = __builtin_ctzll(who);
        const int tb = __builtin_amdgcn_readlane(resc ? __builtin_ctz(resc) : 0, b);
        const int i = tb * L + b;
        const RowMax s = scan_row<S>(ch, o, n, i, exact_mode, r);
        const bool mine = r == b;
        slot_put<S>(o.pmx, tb, s.mx, mine);
        slot_put<S>(o.parg, tb, s.arg, mine);
        if (mine) resc &= resc - 1;
    }
}

// ---- clearance pairs ------------------------------------------------------------------------

// Row ci of the non-zero bit matrix from scratch (the lanes share the objects).
template <int S>
__device__ __forceinline__ void nz_row(const DeltaPtrs& ch, Own<S>& o, int n, int ci, int r) {
    float4 A;  // (ci is wave-uniform)
    if (ci < 64) {
        A.x = grp_get<L>(o.cla0.x, ci, 0);
        A.y = grp_get<L>(o.cla0.y, ci, 0);
        A.z = grp_get<L>(o.cla0.z, ci, 0);
        A.w = grp_get<L>(o.cla0.w, ci, 0);
    } else {
        A = ch.CLA[ci - 64];
    }
#pragma unroll
    for (int w = 0; w < S; ++w) {
        const int j = w * 64 + r;
        const bool nz = j < n && overlap(A, obj_box(ch, j)) != 0.0f;
        const uint64_t word = __ballot(nz);
        if (ci < 64) {
            if (r == ci) o.nz0[w] = word;
        } else if (r == 0) {
            stage(ch.NZ).put((ci - 64) * S + w, word);
        }
    }
}

// Clearance boxes and pair bits after objects ka, kb changed (also restores them after a
// rejected proposal has put the old poses back). Returns whether this lane's first row
// (clearance r < 64) may have changed: its clearance moved, or it pairs with ka or kb before or
// after (the row's cached sums, ClRow, must then be recomputed).
template <int S>
__device__ __forceinline__ bool clearance_delta(const DeltaPtrs& ch, Own<S>& o, int n, int c,
                                                int ka, int kb, int r) {
    if (ka < 0 && kb < 0) return false;
    bool chg0 = false;
    uint64_t rows = 0;
    int t = 0;
    for (int ci = r; ci < c; ci += L, ++t) {
        const int src = ch.clrs[ci].pad;
        if (src == ka || src == kb) {
            cla_put<S>(ch, o, ci, cla_box(ch, ci));
            rows |= 1ull << t;
        }
    }
    chg0 = (rows & 1ull) != 0;  // (a moved row is rebuilt below)
    hand_off(ch.CLA);  // the moved clearances' boxes (64 and up: LDS)
    // Columns ka, kb of the rows whose clearance did not move (lane-owned rows).
    for (int s2 = 0; s2 < 2; ++s2) {
        const int j = s2 == 0 ? ka : kb;
        if (j < 0) continue;
        const float4 bj = obj_box(ch, j);
        const uint64_t bit = 1ull << (j & 63);
        t = 0;
        for (int ci = r; ci < c; ci += L, ++t) {
            if (rows & (1ull << t)) continue;
            const bool nz = overlap(cla_get<S>(ch, o, ci), bj) != 0.0f;
            if (t == 0) {
                const int wj = j >> 6;  // (selects: no dynamic register indexing)
                uint64_t w0 = 0;
#pragma unroll
                for (int q = 0; q < S; ++q) w0 = q == wj ? o.nz0[q] : w0;
                chg0 = chg0 || nz || (w0 & bit) != 0;
                const uint64_t w1 = nz ? (w0 | bit) : (w0 & ~bit);
#pragma unroll
                for (int q = 0; q < S; ++q) o.nz0[q] = q == wj ? w1 : o.nz0[q];
            } else {
                uint64_t* wd = stage(ch.NZ).ptr() + (ci - 64) * S + (j >> 6);
                *wd = nz ? (*wd | bit) : (*wd & ~bit);
            }
        }
    }
    // Rows of the clearances that moved, one at a time.
    for (;;) {
        const uint64_t who = __ballot(rows != 0);
        if (who == 0) break;
        const int b = __builtin_ctzll(who);
        const int tb = __builtin_amdgcn_readlane(rows ? __builtin_ctzll(rows) : 0, b);
        nz_row<S>(ch, o, n, tb * L + b, r);
        if (r == b) rows &= rows - 1;
    }
    return chg0;
}

// The relationship terms a proposal overwrote, so that an undo swaps them back instead of
// evaluating them again (a double atan2, a root and two divisions per relationship): up to two
// per lane (a move touches a handful of relationships), each with its slot t (relationship
// t * L + r). A swap, so a second undo re-applies the proposal's terms (the rare exact pass of
// the current configuration). A lane with more touched relationships sets `all`: the undo then
// evaluates them again.
struct RelBk {
    double pw[2], ang[2];
    int slot[2];
    int cnt;
    bool all;
};

// Terms the plain step holds as fp32 estimates (mh_common.h rel_pw_est, rel_ang_est, cph_est;
// the full kernel's scheme, §4 of DESIGN.md): this lane's objects t * L + r (bit t of `obj`) and
// its relationships in slots u < 2 (bit u of `rel`, q = u * L + r), with the angle estimates'
// allowances. The rejection bound adds their allowances; fix_estimates() makes every one exact
// before a replay. An undo swaps the record back with the terms (a second undo re-applies it).
struct EstState {
    unsigned obj, rel;
    float eang[2];
};

// PairWise / PairWiseAngle terms of the relationships touching ka or kb (or all, ka = -2).
// The hit test reads the relationship objects from LDS; the records themselves (ranges,
// normalisers) come from HBM, for the few relationships a move touches. `bk`: the overwritten
// terms are kept there (the proposal's update).
__device__ __forceinline__ void rels_delta(const DeltaPtrs& ch, int nr, int ka, int kb, int r,
                                           RelBk* bk = nullptr, EstState* est = nullptr) {
    uint64_t pend = 0;
    int t = 0;
    for (int q = r; q < nr; q += L, ++t) {
        const uint2 w = ch.rel[q];
        const int s0 = (int)(w.x & 0xffffu), t0 = (int)(w.x >> 16);
        const int s1 = (int)(w.y & 0xffffu), t1 = (int)(w.y >> 16);
        const bool hit = ka == -2 || s0 == ka || t0 == ka || s1 == ka || t1 == ka ||
                         (kb >= 0 && (s0 == kb || t0 == kb || s1 == kb || t1 == kb));
        if (hit) pend |= 1ull << t;
    }
    if (bk) {
        bk->cnt = 0;
        bk->all = __builtin_popcountll(pend) > 2;
    }
    while (__ballot(pend != 0)) {
        if (pend) {
            const int u = __builtin_ctzll(pend);
            const int q = u * L + r;
            pend &= pend - 1;
            if (bk && bk->cnt < 2) {
                const int k = bk->cnt;
                const double p = ch.RPW[q], g = ch.RANG[q];
                if (k == 0) {  // (constant indices: registers, not scratch)
                    bk->pw[0] = p;
                    bk->ang[0] = g;
                    bk->slot[0] = u;
                } else {
                    bk->pw[1] = p;
                    bk->ang[1] = g;
                    bk->slot[1] = u;
                }
                bk->cnt = k + 1;
            }
            double tpw, tang;
            bool amb = true;  // (no estimate: the exact terms)
            if (est && u < 2) {  // the plain step: fp32 estimates with allowances
                const uint2 w = ch.rel[q];
                const ObjP ps = obj_pose(ch, (int)(w.x & 0xffffu)), pt = obj_pose(ch, (int)(w.x >> 16));
                const ObjP as = obj_pose(ch, (int)(w.y & 0xffffu)), atp = obj_pose(ch, (int)(w.y >> 16));
                const float4 e0 = ch.rele[q], e1 = ch.rele[ch.nre + q];
                amb = false;
                tpw = rel_pw_est(e0, ps, pt, amb);
                const float ay = as.yf - atp.yf, ax = as.xf - atp.xf;
                amb |= !(fmaxf(fabsf(ay), fabsf(ax)) >= 0x1p-100f);
                float ea = 0.0f;
                tang = rel_ang_est(e1, e0.w, atp, atan2_est(ay, ax), ea, amb);
                const unsigned bit = 1u << u;
                est->rel = amb ? (est->rel & ~bit) : (est->rel | bit);
                if (u == 0) est->eang[0] = ea;
                else est->eang[1] = ea;
            }
            if (amb) rel_terms_of(ch.relg[q], [&ch](int k) { return obj_pose(ch, k); }, tpw, tang);
            stage(ch.RPW).put(q, -tpw);
            stage(ch.RANG).put(q, -tang);
        }
    }
}

// Undo of rels_delta's proposal update: the kept terms swapped back (or, where a lane's record
// is incomplete, the touched relationships evaluated again).
__device__ __forceinline__ void rels_undo(const DeltaPtrs& ch, int nr, int ka, int kb, int r,
                                          RelBk& bk) {
    if (__ballot(bk.all)) {
        rels_delta(ch, nr, ka, kb, r);
        return;
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (k < bk.cnt) {
            const int q = bk.slot[k] * L + r;
            const double p = ch.RPW[q], g = ch.RANG[q];
            stage(ch.RPW).put(q, bk.pw[k]);
            stage(ch.RANG).put(q, bk.ang[k]);
            bk.pw[k] = p;
            bk.ang[k] = g;
        }
    }
}

// ---- compacted Clearance / SurfaceArea terms ------------------------------------------------

// The rejection bound's Clearance terms of this lane's first row (clearance r < 64): their
// negated sum in the row's order, their count, and the sum of in-row position x |term|. Kept per
// configuration and recomputed only for rows a proposal may change (clearance_delta), so a step
// the bound decides builds no Clearance list. (Rooms of more than 64 clearances use the list
// build for the bound, as the rows past 64 are not cached.)
struct ClRow {
    float sum;
    int cnt;
    float pos;
};

template <int S>
__device__ __forceinline__ ClRow cl_row0(const DeltaPtrs& ch, const Own<S>& o, int c, int r,
                                         bool active) {
    ClRow w{0.0f, 0, 0.0f};
    if (active && r < c) {
        const float4 A = o.cla0;
#pragma unroll
        for (int q = 0; q < S; ++q) {
            uint64_t word = o.nz0[q];
            while (word) {
                const int j = q * 64 + __builtin_ctzll(word);
                word &= word - 1;
                const float v = -overlap(A, obj_box(ch, j));
                w.sum += v;
                w.pos = fmaf((float)w.cnt, -v, w.pos);
                ++w.cnt;
            }
        }
    }
    return w;
}

// Non-zero Clearance terms, clearance-major then object (Kernel.cu:408-431), negated: those at
// positions [lo, lo + cap_cl) go to LCL[pos - lo]. Returns the total count. With `sum`, also
// this lane's partial sum of the terms it evaluated and their count (the rejection bound).
template <int S>
__device__ __forceinline__ int build_cl_list(const DeltaPtrs& ch, const Own<S>& o, int c, int r,
                                             int lo, float* sum = nullptr,
                                             int* cnt_own = nullptr, float* possum = nullptr) {
    int base = 0;
    float acc = 0.0f, accp = 0.0f;  // (accp: sum of pos |term|, the bound's position weights)
    int own = 0;
    for (int cb = 0; cb < c; cb += L) {
        const int ci = cb + r;
        uint64_t wd[S];
#pragma unroll
        for (int w = 0; w < S; ++w)
            wd[w] = ci >= c ? 0ull : (cb == 0 ? (uint64_t)o.nz0[w] : ch.NZ[(ci - 64) * S + w]);
        int cnt = 0;
#pragma unroll
        for (int w = 0; w < S; ++w) cnt += __builtin_popcountll(wd[w]);
        int tot;
        int pos = base + group_excl_scan<L>(cnt, r, tot);
        own += cnt;
        if (cnt) {
            const float4 A = cla_get<S>(ch, o, ci);
#pragma unroll
            for (int w = 0; w < S; ++w) {
                uint64_t word = wd[w];
                while (word) {
                    const int j = w * 64 + __builtin_ctzll(word);
                    word &= word - 1;
                    const float v = -overlap(A, obj_box(ch, j));
                    acc += v;
                    accp = fmaf((float)pos, -v, accp);
                    if (pos >= lo && pos < lo + ch.cap_cl) stage(ch.LCL).put(pos - lo, v);
                    ++pos;
                }
            }
        }
        base += tot;
    }
    if (sum) {
        *sum = acc;
        *cnt_own = own;
        *possum = accp;
    }
    return base;
}

// Non-zero SurfaceArea terms in the reference's order, negated: positions [lo, lo + cap_sa) go
// to LSA[pos - lo]. Returns the total count. With `sum`, this lane's partial sum of its terms.
__device__ __forceinline__ int build_sa_list(const DeltaPtrs& ch, int n, int c, int r, int lo,
                             float* sum = nullptr) {
    int base = 0;
    float acc = 0.0f;
    const int ne = c + n;
    for (int eb = 0; eb < ne; eb += L) {
        const int e = eb + r;
        const bool set = e < ne && ((ch.SAM[e >> 5] >> (e & 31)) & 1u);
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        int cnt = 0;
        if (set) {
            v = sa_entry(ch, c, e);
            cnt = (v.x != 0.0f) + (v.y != 0.0f) + (v.z != 0.0f) + (v.w != 0.0f);
            acc -= (v.x + v.y) + (v.z + v.w);
        }
        int tot;
        int pos = base + group_excl_scan<L>(cnt, r, tot);
        if (cnt) {
            const float tv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (tv[u] != 0.0f) {
                    if (pos >= lo && pos < lo + ch.cap_sa) stage(ch.LSA).put(pos - lo, -tv[u]);
                    ++pos;
                }
        }
        base += tot;
    }
    if (sum) *sum = acc;
    return base;
}

// ---- terms for the rejection bound (certain_reject, mh_common.h) --------------------------

// This lane's partial sums of the dense terms of Costs() for the configuration in LDS: its
// objects (VisualBalance, FocalPoint, the proposed Symmetry rows) and its relationships. The
// Clearance and SurfaceArea partial sums come from the list builds (build_cl_list /
// build_sa_list), which write the lists as they go.
template <int S>
__device__ __forceinline__ BoundTerms delta_bound_terms(const DeltaPtrs& ch, const Own<S>& o, int n, int c,
                                        int nr, int r, const EstState& est) {
    BoundTerms bt;
    bt.nx = bt.ny = bt.anx = bt.any = bt.fp = bt.afp = bt.sym = bt.cl = bt.sa = 0.0f;
    bt.symw = bt.clpos = 0.0f;
    bt.pw = bt.ang = bt.aang = 0.0f;
    bt.pwd = bt.angd = 0.0;
    bt.efp = bt.eang = bt.esym = 0.0f;  // (exact terms only)
    bt.pwx = 0;
#pragma unroll
    for (int t = 0; t < S; ++t) {
        const int i = t * L + r;
        if (i < n) {
            const float a = ch.AREA[i];
            const float tx = (float)((double)a * ch.X[i]), ty = (float)((double)a * ch.Y[i]);
            bt.nx += tx;
            bt.ny += ty;
            bt.anx += fabsf(tx);
            bt.any += fabsf(ty);
            const float w = ch.CPH[i];
            bt.fp += w;
            bt.afp += fabsf(w);
            bt.sym -= o.pmx[t];
            bt.symw = fmaf((float)(n - i), o.pmx[t], bt.symw);  // (row i: position i)
        }
    }
    for (int q = r; q < nr; q += L) {  // (summed in double: bound_decide<true>)
        const double tp = ch.RPW[q], ta = ch.RANG[q];
        bt.pwd += tp;
        bt.angd += ta;
        bt.aang += fabsf((float)ta);
    }
    bt.k = max(max((n + L - 1) / L, (nr + L - 1) / L), 4 * ((c + n + L - 1) / L));  // uniform
    // the estimated terms' allowances (EstState): FocalPoint kDeltaCph each, PairWise kPwEstU U
    // relative (uniform), PairWiseAngle eang each
    bt.efp = kDeltaCph * (float)__builtin_popcount(est.obj);
    bt.eang = ((est.rel & 1u) ? est.eang[0] : 0.0f) + ((est.rel & 2u) ? est.eang[1] : 0.0f);
    bt.pwx = __ballot(est.rel != 0u) ? kPwEstU : 0;
    return bt;
}

// ---- proposal (propose(), Kernel.cu:566-704) in place ---------------------------------------

// Object k's pose (wave-uniform k).
template <int S>
__device__ __forceinline__ DBackup read_obj(const DeltaPtrs& ch, const Own<S>& o, int k) {
    DBackup b;
    b.k = k;
    b.w = ch.CPH[k];
    b.x = ch.X[k];
    b.y = ch.Y[k];
    b.ry = obj_ry<S>(o, k);
    return b;
}

// New pose of object k (its FocalPoint term is refreshed separately): LDS (with its box) by
// `writer`, the owner lane's registers.
template <int S>
__device__ __forceinline__ void write_pose(const DeltaPtrs& ch, Own<S>& o, int r, bool writer,
                                           int k, double x, double y, double ry) {
    if (writer) {
        stage(ch.X).put(k, x);
        stage(ch.Y).put(k, y);
        stage(ch.BOX).put(k, shape_box(ch.objs[k], (float)x, (float)y));
        stage(ch.RYF).put(k, (float)ry);
    }
    const bool own = r == (k & 63);
    slot_put<S>(o.ry, k >> 6, ry, own);
    slot_put<S>(o.xf, k >> 6, (float)x, own);
    slot_put<S>(o.yf, k >> 6, (float)y, own);
}

template <int S, class Rng>
__device__ __forceinline__ int2 propose(Rng& rng, const DevRoom& rm, const unsigned char* frozen,
                        const DeltaPtrs& ch, Own<S>& o, int r, bool writer) {
    const int n = rm.n;
    const int mode = rand_int(rng, 2, 0);
    if (mode == 0) {  // translate, Kernel.cu:595-632
        const int k = pick_object(rng, n, frozen);
        float dx = rng.normal();
        dx = dx * rm.sx;
        float dy = rng.normal();
        dy = dy * rm.sy;
        const DBackup b0 = read_obj<S>(ch, o, k);
        double x = b0.x, y = b0.y;
        if (x + (double)dx > rm.rmax_x) x = rm.rmax_x;
        else if (x + (double)dx < rm.rmin_x) x = rm.rmin_x;
        else x = x + (double)dx;
        if (y + (double)dy > rm.rmax_y) y = rm.rmax_y;
        else if (y + (double)dy < rm.rmin_y) y = rm.rmin_y;
        else y = y + (double)dy;
        if (writer) {
            const Staged<DeltaAux> ax = stage(ch.aux);
            ax->b[0] = b0;
            ax->nb = 1;
            ax->swap_a = -1;
        }
        write_pose<S>(ch, o, r, writer, k, x, y, b0.ry);
        return make_int2(k, -1);
    }
    if (mode == 1) {  // rotate, Kernel.cu:634-653
        const int k = pick_object(rng, n, frozen);
        float dr = rng.normal();
        dr = (float)((double)dr * kSigmaT);
        const DBackup b0 = read_obj<S>(ch, o, k);
        double ry = b0.ry + (double)dr;
        if (ry < 0) ry = ry + kTwoPI;
        else if (ry > kTwoPI) ry = ry - kTwoPI;
        if (writer) {
            const Staged<DeltaAux> ax = stage(ch.aux);
            ax->b[0] = b0;
            ax->nb = 1;
            ax->swap_a = -1;
        }
        write_pose<S>(ch, o, r, writer, k, b0.x, b0.y, ry);
        return make_int2(k, -1);
    }
    // swap, Kernel.cu:655-703: object 1's pose travels through float temporaries.
    if (n < 2) {
        if (writer) {
            const Staged<DeltaAux> ax = stage(ch.aux);
            ax->nb = 0;
            ax->swap_a = -1;
        }
        return make_int2(-1, -1);
    }
    const int ka = pick_object(rng, n, frozen);
    const int kb = pick_object(rng, n, frozen);
    const DBackup b0 = read_obj<S>(ch, o, ka);
    const DBackup b1 = read_obj<S>(ch, o, kb);
    if (writer) {
        const Staged<DeltaAux> ax = stage(ch.aux);
        ax->b[0] = b0;
        ax->b[1] = b1;
        ax->nb = 2;
        ax->swap_a = ka;
        ax->swap_b = kb;
    }
    write_pose<S>(ch, o, r, writer, ka, b1.x, b1.y, b1.ry);
    write_pose<S>(ch, o, r, writer, kb, (double)(float)b0.x, (double)(float)b0.y,
                  (double)(float)b0.ry);
    return make_int2(ka, kb == ka ? -1 : kb);
}

__device__ __forceinline__ void commit_swap_zrr(const DeltaPtrs& ch, int n) {
    const int ka = ch.aux->swap_a, kb = ch.aux->swap_b;
    if (ka < 0) return;
#pragma unroll
    for (int f = 0; f < 3; ++f) {
        double* row = ch.zrr + f * n;
        const double va = row[ka], vb = row[kb];
        row[ka] = vb;
        row[kb] = (double)(float)va;
    }
}

// Saves the proposed configuration (cfgStar, Kernel.cu:810-811) to the chain's best slot: lane
// r writes its objects; z, rotX, rotZ come from HBM with a pending swap applied as
// commit_swap_zrr would (ka takes kb's values, kb takes ka's rounded to float).
template <int S>
__device__ __forceinline__ void save_best_delta(const DeltaPtrs& ch, const Own<S>& o,
                                                double* dst, int n, int r) {
    const int ka = ch.aux->swap_a, kb = ch.aux->swap_b;
#pragma unroll
    for (int t = 0; t < S; ++t) {
        const int i = t * L + r;
        if (i >= n) break;
        dst[F_X * n + i] = ch.X[i];
        dst[F_Y * n + i] = ch.Y[i];
        dst[F_RY * n + i] = o.ry[t];
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

// ---- the ordered sums (Costs(), Kernel.cu:516-549) -----------------------------------------

// Lane k < 8 of the chain walks sum k in the reference's order from the cached terms: 0/1
// VisualBalance area*x, area*y (double terms, float accumulators, :200-201); 2 FocalPoint
// (float terms, double accumulator, :277); 3 Symmetry (float, float, :314); 4 Clearance and
// 5 SurfaceArea (float, float); 6/7 PairWise and PairWiseAngle (double, double). Each step is
// rn_d(acc + v) with v the (negated where the reference subtracts) term, rounded on to float
// for the float accumulators. Every lane reads three streams -- multiplier m, double d, float f
// -- and adds v = m * d + f;
// the streams a sum does not use are ones or zeros, and each sequence is zero past its end, so
// v is the reference's term exactly.
// Sums list terms [from, to) of `fs` (the float list of lane k = 4 or 5) into the float
// accumulator a, four at a time: the reference's float accumulator with float terms, so the
// double-rounded add of the dense walk equals the plain fp32 add (53 >= 2 * 24 + 2 bits). The
// entries up to round4(to) are zero (x + 0 == x).
// The next four terms are loaded before the current four are added, so the LDS latency
// overlaps the dependent adds (these walks run ~1,000 terms at N = 256 on few waves per SIMD).
__device__ __forceinline__ float list_walk(const float* fs, int from, int to, float a) {
    if (from >= to) return a;
    float4 q = load16<float4>(fs + from);
    for (int l = from; l < to; l += 4) {
        const float4 nq = (l + 4 < to) ? load16<float4>(fs + l + 4) : q;
        a = a + q.x;
        a = a + q.y;
        a = a + q.z;
        a = a + q.w;
        q = nq;
    }
    return a;
}

// (`dense`: diagnostic builds add the cycles of the dense walk to it)
template <int S>
__device__ __forceinline__ void replay(const DeltaPtrs& ch, const Own<S>& o, int n, int cnt_cl,
                                       int cnt_sa, int r, float out[8],
                                       unsigned long long* dense = nullptr) {
#if MH_STAMPS
    unsigned long long t_in;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_in) :: "memory");
#endif
    const DevRoom& rm = *ch.rm;
    const int k = r;
    // Each lane's three streams (multiplier, double, float); a stream a sum does not use, and
    // every stream past its end, reads ones or zeros, each typed as read: ch.ONES and ch.ZERO (DL
    // entries) and ch.ZEROF (four float zeros the float pointer does not advance over).
    const float* ms = ch.ONES;
    const double* ds = ch.ZERO;
    const float* fs = ch.ZEROF;
    bool fstream = false;
    int lim = ch.NP;  // this lane's stream length; past it the lane reads ones / zeros
    if (k < 2) {
        ms = ch.AREA;
        ds = k == 0 ? ch.X.ptr() : ch.Y.ptr();
    } else if (k == 2) {
        fs = ch.CPH.ptr();
        fstream = true;
    } else if (k == 3) {
        fs = ch.NMX.ptr();
        fstream = true;
    } else if (k == 4) {
        fs = ch.LCL.ptr();
        fstream = true;
    } else if (k == 5) {
        fs = ch.LSA.ptr();  // (its capacity may be below NP: the stream ends at the zero-filled end)
        fstream = true;
        lim = (min(cnt_sa, ch.cap_sa) + 3) & ~3;
    } else if (k == 6) {
        ds = ch.RPW.ptr();
        lim = ch.NR;
    } else if (k == 7) {
        ds = ch.RANG.ptr();
        lim = ch.NR;
    }
    double accf = 0.0, accd = 0.0;  // float- and double-accumulated walks of the same terms
    for (int l0 = 0; l0 < ch.DL; l0 += 4) {
        const bool in = l0 < lim;
        const float* msl = in ? ms : ch.ONES;
        const double* dsl = in ? ds : ch.ZERO;
        const float* fsl = in && fstream ? fs + l0 : ch.ZEROF;
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            // one rounding either way: rn(m * d) where f = 0 (VisualBalance: m = area) and
            // rn(d + f) where m = 1 (every other sum), so the fused form is the two-step one
            v[u] = __builtin_fma((double)msl[l0 + u], dsl[l0 + u], (double)fsl[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            accd = accd + v[u];
            accf = (double)(float)(accf + v[u]);
        }
    }
#if MH_STAMPS
    {
        __builtin_amdgcn_sched_barrier(0);
        unsigned long long t_out;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_out) :: "memory");
        if (dense) *dense += t_out - t_in;
        __builtin_amdgcn_sched_barrier(0);
    }
#endif
    // Clearance / SurfaceArea lists longer than NP: their tails, then (lists longer than the
    // buffer, rare) further windows rebuilt in place.
    const int cnt = k == 4 ? cnt_cl : (k == 5 ? cnt_sa : 0);
    const int cap = k == 4 ? ch.cap_cl : ch.cap_sa;
    float af = (float)accf;
    const int tail = (min(cnt, cap) + 3) & ~3;
    const int walked = min(lim, ch.DL);  // what the dense walk covered of this lane's stream
    if (tail > walked) af = list_walk(fs, walked, tail, af);
    for (int lo = ch.cap_cl; lo < cnt_cl; lo += ch.cap_cl) {
        hand_off(ch.LCL);  // (the previous window's walk is done before the list is rebuilt)
        build_cl_list<S>(ch, o, rm.c, r, lo);
        const int m = min(ch.cap_cl, cnt_cl - lo);
        for (int l = m + r; l < ((m + 3) & ~3); l += L) stage(ch.LCL).put(l, 0.0f);
        hand_off(ch.LCL);  // the window, to its walking lane
        if (k == 4) af = list_walk(ch.LCL.ptr(), 0, (m + 3) & ~3, af);
    }
    for (int lo = ch.cap_sa; lo < cnt_sa; lo += ch.cap_sa) {
        hand_off(ch.LSA);
        build_sa_list(ch, n, rm.c, r, lo);
        const int m = min(ch.cap_sa, cnt_sa - lo);
        for (int l = m + r; l < ((m + 3) & ~3); l += L) stage(ch.LSA).put(l, 0.0f);
        hand_off(ch.LSA);
        if (k == 5) af = list_walk(ch.LSA.ptr(), 0, (m + 3) & ~3, af);
    }
    accf = (double)af;
    const bool acc_float = (k == 0 || k == 1 || k == 3 || k == 4 || k == 5);
    const double acc = acc_float ? accf : accd;
    const float nx = (float)grp_get<L>(acc, 0, 0);
    const float ny = (float)grp_get<L>(acc, 1, 0);
    const double fp = grp_get<L>(acc, 2, 0);
    const float sym = (float)grp_get<L>(acc, 3, 0);
    const float cl = (float)grp_get<L>(acc, 4, 0);
    const float sa = (float)grp_get<L>(acc, 5, 0);
    const double pw = grp_get<L>(acc, 6, 0);
    const double ang = grp_get<L>(acc, 7, 0);
    const float vb = (float)(-1.0 * distance_f(nx / rm.denom, ny / rm.denom, rm.cxf, rm.cyf));
    const float pwc = (float)(pw * ang);
    out[1] = rm.w_pw * pwc;
    out[2] = rm.w_vb * vb;
    out[3] = rm.w_fp * (float)fp;
    out[4] = rm.w_sym * sym;
    out[6] = rm.w_ol * 0.0f;  // OffLimits never enters the step (Kernel.cu:547)
    out[5] = rm.w_cl * cl;
    out[7] = rm.w_sa * sa;
    float t = out[1] + out[2];
    t = t + out[3];
    t = t + out[4];
    t = t + out[5];
    t = t + out[7];
    out[0] = t;
}

// Chains (waves) per workgroup the kernel is built for: rooms of more than 128 objects are held
// by LDS to at most two chains per SIMD, so a bound of eight lets the allocator use up to 256
// VGPRs (twelve would cap it at 168 and spill).
constexpr int delta_max_waves_s(int S) { return S >= 4 ? 8 : 12; }

// The exact costs of the configuration the caches hold, with symmetry rows `mx` (the proposal's
// o.pmx or the current o.cmx), from the Clearance / SurfaceArea lists just built (counts cnt_cl,
// cnt_sa): zero past each list's end, the Symmetry stream, the replay.
template <int S>
__device__ __forceinline__ void replay_config(const DeltaPtrs& ch, const typename Own<S>::fvec& mx,
                                              const Own<S>& o, int n, int cnt_cl, int cnt_sa,
                                              int r, float out[8],
                                              unsigned long long* dense = nullptr) {
    // zero past each list's end: to NP for the dense walk, to round4 for the list walk
    const int zcl = max(ch.NP, (min(cnt_cl, ch.cap_cl) + 3) & ~3);
    const int zsa = (min(cnt_sa, ch.cap_sa) + 3) & ~3;  // (lane 5's dense stream ends there)
    for (int l = min(cnt_cl, ch.cap_cl) + r; l < zcl; l += L) stage(ch.LCL).put(l, 0.0f);
    for (int l = min(cnt_sa, ch.cap_sa) + r; l < zsa; l += L) stage(ch.LSA).put(l, 0.0f);
#pragma unroll
    for (int t = 0; t < S; ++t) {
        const int i = t * L + r;
        if (i < n) stage(ch.NMX).put(i, -mx[t]);
    }
    // the replay's streams, as their lanes walk them
    hand_off(ch.X, ch.Y, ch.CPH, ch.NMX, ch.LCL, ch.LSA, ch.RPW, ch.RANG);
    replay<S>(ch, o, n, cnt_cl, cnt_sa, r, out, dense);
}

// Makes every estimated term of this lane exact (EstState): the objects' FocalPoint terms and
// the slots' relationship terms, evaluated as the reference does; check builds verify each
// estimate against its allowance first (sites 30-32, as in the full kernel).
template <int S>
__device__ __forceinline__ void fix_estimates(const DeltaPtrs& ch, const Own<S>& o, EstState& est,
                                              int r) {
#pragma unroll
    for (int t = 0; t < S; ++t) {
        const bool b = ((est.obj >> t) & 1u) != 0;
        if (__ballot(b) && b) {
            const int i = t * L + r;
            const float w = focal_cos(*ch.rm, o.xf[t], o.yf[t], (float)o.ry[t]);
            MH_CK(fabsf(-ch.CPH[i] - w) <= kDeltaCph, 30, __float_as_uint(-ch.CPH[i]),
                  __float_as_uint(w));
            stage(ch.CPH).put(i, -w);
        }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const bool b = ((est.rel >> u) & 1u) != 0;
        if (__ballot(b) && b) {
            const int q = u * L + r;
            double tpw, tang;
            rel_terms_of(ch.relg[q], [&ch](int k) { return obj_pose(ch, k); }, tpw, tang);
            MH_CK(fabs(-ch.RPW[q] - tpw) <= kPwEstU * 0x1p-24 * fabs(tpw) + 1e-30, 31,
                  __float_as_uint((float)-ch.RPW[q]), __float_as_uint((float)tpw));
            MH_CK(fabs(-ch.RANG[q] - tang) <= (double)est.eang[u], 32,
                  __float_as_uint((float)-ch.RANG[q]), __float_as_uint((float)tang));
            stage(ch.RPW).put(q, -tpw);
            stage(ch.RANG).put(q, -tang);
        }
    }
    est.obj = est.rel = 0u;
    hand_off(ch.CPH, ch.RPW, ch.RANG);  // the exact terms
}

// Undoes the last proposal (objects ka, kb): the backed-up poses and FocalPoint terms, the
// SurfaceArea bits (SAM <-> SAMB, so the proposal's bits stay in SAMB), the clearance boxes and
// pair bits, the relationship terms.
template <int S>
__device__ __forceinline__ void undo_proposal(const DeltaPtrs& ch, Own<S>& o, int n, int c, int nr,
                                              int ka, int kb, int r, bool writer, RelBk& rbk,
                                              typename Own<S>::wvec& bk_nz, EstState& est,
                                              EstState& est_bk) {
    {  // the estimate record of the terms restored below (a swap, as the terms)
        const EstState t = est;
        est = est_bk;
        est_bk = t;
    }
    const int nb = ch.aux->nb;
    for (int q = nb - 1; q >= 0; --q) {
        const DBackup b = ch.aux->b[q];
        write_pose<S>(ch, o, r, writer, b.k, b.x, b.y, b.ry);
        if (writer) stage(ch.CPH).put(b.k, b.w);
    }
    for (int w = r; w < ch.SW; w += L) {
        const uint32_t t = ch.SAM[w];
        stage(ch.SAM).put(w, ch.SAMB[w]);
        stage(ch.SAMB).put(w, t);
    }
    // the restored poses, boxes, FocalPoint terms and SurfaceArea bits
    hand_off(ch.X, ch.Y, ch.BOX, ch.RYF, ch.CPH, ch.SAM, ch.SAMB);
    // The Clearance row words the proposal overwrote in registers (clearances < 64) are swapped
    // back, not recomputed (a swap: a second undo re-applies the proposal's), and a clearance
    // whose source moved takes its box at the restored pose; rooms of more than 64 clearances,
    // whose further rows live in LDS, recompute.
    if (c <= 64) {
        const typename Own<S>::wvec w = o.nz0;
        o.nz0 = bk_nz;
        bk_nz = w;
        const bool moved = r < c && (ch.clrs[r].pad == ka || ch.clrs[r].pad == kb);
        if (__ballot(moved))
            if (moved) o.cla0 = cla_box(ch, r);
    } else {
        clearance_delta<S>(ch, o, n, c, ka, kb, r);
    }
    rels_undo(ch, nr, ka, kb, r, rbk);
    hand_off(ch.CLA, ch.NZ, ch.RPW, ch.RANG);  // the restored pairs and relationship terms
}

// ---- the kernel ---------------------------------------------------------------------------

template <int S, bool XW, bool TRACK>
// Up to 12 waves (chains) per workgroup: at large N one workgroup per CU holds every resident
// chain, so the room tables staged in LDS are paid for once per CU (three waves per SIMD leave
// the register allocator 168 registers).
__global__ void __launch_bounds__(64 * delta_max_waves_s(S)) mh_delta_kernel(LaunchArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const DeltaLds& lay = a.dlay;
    const int n = a.rm.n, c = a.rm.c, nr = a.rm.r;
    const int r = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int waves_per_wg = blockDim.x >> 6;

    RectShape* objs_l = reinterpret_cast<RectShape*>(lds + lay.h_obj);
    RectShape* clrs_l = reinterpret_cast<RectShape*>(lds + lay.h_clr);
    uint2* rel_l = reinterpret_cast<uint2*>(lds + lay.h_rel);
    unsigned char* frozen = lds + lay.h_frz;
    DevRoom* rm_l = reinterpret_cast<DevRoom*>(lds + lay.h_room);
    for (int i = threadIdx.x; i < n; i += blockDim.x) objs_l[i] = a.objc[i].off;
    for (int i = threadIdx.x; i < c; i += blockDim.x) {
        RectShape cs = a.clrc[i].shape;
        cs.pad = a.clrc[i].src;
        clrs_l[i] = cs;
    }
    for (int i = threadIdx.x; i < nr; i += blockDim.x)
        rel_l[i] = make_uint2((unsigned)a.relc[i].s | ((unsigned)a.relc[i].t << 16),
                              (unsigned)a.relc[i].as | ((unsigned)a.relc[i].at << 16));
    for (int i = threadIdx.x; i <= n; i += blockDim.x) frozen[i] = (i < n) ? (a.objc[i].frozen != 0) : 1;
    if (threadIdx.x == 0) *rm_l = a.rm;
    {
        float* area = reinterpret_cast<float*>(lds + lay.h_area);
        float* ones = reinterpret_cast<float*>(lds + lay.h_ones);
        double* zero = reinterpret_cast<double*>(lds + lay.h_zero);
        float* zerof = reinterpret_cast<float*>(lds + lay.h_zero + round16(8 * lay.DL));  // 4
        for (int i = threadIdx.x; i < lay.DL; i += blockDim.x) {
            area[i] = i < n ? a.objc[i].area : 0.0f;
            ones[i] = 1.0f;
            zero[i] = 0.0;
        }
        if (threadIdx.x < 4) zerof[threadIdx.x] = 0.0f;
    }
    __syncthreads();

    const int64_t chain = (int64_t)blockIdx.x * waves_per_wg + wave;
    if (chain >= a.n_chains) return;

    // The per-chain LDS addresses are computed into VGPRs (an opaque v_mov), not kept in SGPRs:
    // this kernel is bound by LDS per chain, not registers, and the scalar file was spilling.
    int boff = lay.hdr + wave * lay.stride;
    asm volatile("v_mov_b32 %0, %1" : "=v"(boff) : "v"(boff));
    unsigned char* base = lds + boff;
    DeltaPtrs ch;
    ch.objs = objs_l;
    ch.clrs = clrs_l;
    ch.rel = rel_l;
    ch.relg = a.relc;
    ch.rele = a.rele;
    ch.nre = nr > 0 ? nr : 1;
    ch.rm = rm_l;
    ch.AREA = reinterpret_cast<const float*>(lds + lay.h_area);
    ch.ONES = reinterpret_cast<const float*>(lds + lay.h_ones);
    ch.ZERO = reinterpret_cast<const double*>(lds + lay.h_zero);
    ch.ZEROF = reinterpret_cast<const float*>(lds + lay.h_zero + round16(8 * lay.DL));
    ch.X = {reinterpret_cast<double*>(base + lay.X)};
    ch.Y = {reinterpret_cast<double*>(base + lay.Y)};
    ch.BOX = {reinterpret_cast<float4*>(base + lay.BOX)};
    ch.RYF = {reinterpret_cast<float*>(base + lay.RYF)};
    ch.CPH = {reinterpret_cast<float*>(base + lay.CPH)};
    ch.NMX = {reinterpret_cast<float*>(base + lay.NMX)};
    const int np = lay.NP;
    ch.CLA = {reinterpret_cast<float4*>(base + lay.CLA)};
    ch.NZ = {reinterpret_cast<uint64_t*>(base + lay.NZ)};
    ch.SAM = {reinterpret_cast<uint32_t*>(base + lay.SAM)};
    ch.SAMB = {reinterpret_cast<uint32_t*>(base + lay.SAMB)};
    ch.RPW = {reinterpret_cast<double*>(base + lay.RPW)};
    ch.RANG = {reinterpret_cast<double*>(base + lay.RANG)};
    ch.LCL = {reinterpret_cast<float*>(base + lay.LCL)};
    ch.LSA = {reinterpret_cast<float*>(base + lay.LSA)};
    ch.aux = {reinterpret_cast<DeltaAux*>(base + lay.AUX)};
    ch.W = lay.W;
    ch.SW = lay.SW;
    ch.cap_cl = lay.cap_cl;
    ch.cap_sa = lay.cap_sa;
    ch.NP = np;
    ch.NR = lay.NR;
    ch.DL = lay.DL;
    ch.zrr = a.st + chain * (int64_t)(F_COUNT * n) + F_Z * n;
    const int nrp = lay.NR;  // relationship stream length

    // Stage the configuration (rotY into the owner lanes' registers), zero the streams past
    // their ends, build every cache.
    const double* src = a.st + chain * (int64_t)(F_COUNT * n);
    Own<S> o;
#pragma unroll
    for (int t = 0; t < S; ++t) {
        o.ry[t] = 0.0;
        o.xf[t] = o.yf[t] = 0.0f;
        o.cmx[t] = o.pmx[t] = 0.0f;
        o.carg[t] = o.parg[t] = -1;
        o.nz0[t] = 0ull;
        o.cla0 = make_float4(0.f, 0.f, 0.f, 0.f);
        const int i = t * L + r;
        if (i < n) {
            o.ry[t] = src[F_RY * n + i];
            o.xf[t] = (float)src[F_X * n + i];
            o.yf[t] = (float)src[F_Y * n + i];
        }
    }
    for (int i = r; i < np; i += L) {
        double x = 0.0, y = 0.0;
        float ryf = 0.0f;
        float4 box = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < n) {
            x = src[F_X * n + i];
            y = src[F_Y * n + i];
            ryf = (float)src[F_RY * n + i];
            box = shape_box(objs_l[i], (float)x, (float)y);
        }
        stage(ch.BOX).put(i, box);
        stage(ch.RYF).put(i, ryf);
        stage(ch.CPH).put(i, 0.0f);
        stage(ch.X).put(i, x);
        stage(ch.Y).put(i, y);
        stage(ch.NMX).put(i, 0.0f);
    }
    for (int q = r; q < nrp; q += L) {
        stage(ch.RPW).put(q, 0.0);
        stage(ch.RANG).put(q, 0.0);
    }
    for (int w = r; w < ch.SW; w += L) stage(ch.SAM).put(w, 0u);
    // the staged configuration and the streams' zero tails
    hand_off(ch.BOX, ch.RYF, ch.CPH, ch.X, ch.Y, ch.NMX, ch.RPW, ch.RANG, ch.SAM);
    int wild = 0;
#pragma unroll
    for (int t = 0; t < S; ++t) {
        const int i = t * L + r;
        if (i < n) {
            stage(ch.CPH).put(i, -focal_cos(*rm_l, o.xf[t], o.yf[t], (float)o.ry[t]));
            wild += wild_pose(ch.X[i], ch.Y[i], o.ry[t]) ? 1 : 0;
        }
    }
    int wild_cnt = group_sum<L>(wild);
#pragma unroll
    for (int t = 0; t < 2 * S; ++t) {
        const int e = t * L + r;
        o.sav[t] = 0.0f;
        if (e < c + n) {
            const float4 v = sa_entry(ch, c, e);
            if (nonzero4(v)) {
                sam_put(ch, e, true);
                o.sav[t] = (v.x + v.y) + (v.z + v.w);
            }
        }
    }
    for (int ci = r; ci < c; ci += L) cla_put<S>(ch, o, ci, cla_box(ch, ci));
    hand_off(ch.CPH, ch.SAM, ch.CLA);  // FocalPoint terms, SurfaceArea bits, clearance boxes
    for (int ci = 0; ci < c; ++ci) nz_row<S>(ch, o, n, ci, r);
    ClRow rc_cur = cl_row0<S>(ch, o, c, r, true);  // (the current configuration's first rows)
    rels_delta(ch, nr, -2, -1, r);
    for (int i = 0; i < n; ++i) {
        const RowMax s = scan_row<S>(ch, o, n, i, wild_cnt > 0, r);
        slot_put<S>(o.cmx, i >> 6, s.mx, r == (i & 63));
        slot_put<S>(o.carg, i >> 6, s.arg, r == (i & 63));
    }
    hand_off(ch.NZ, ch.RPW, ch.RANG);  // the pair rows and the relationship terms

    const ChainMeta m0 = a.meta[chain];
    const bool writer = r == 0;
    float cur[8];  // resultCosts of the current configuration (wave-uniform: scalar registers)
#pragma unroll
    for (int k = 0; k < 8; ++k) cur[k] = uniform_f(m0.costs[k]);
    float cur_total = m0.costs[0];
    // Plain chains take a proposal the rejection bound certainly accepts without its exact
    // costs: the current total is then known as an interval (cur_iv, cur_exact false) until a
    // step's decision needs it exactly, or the launch ends.
    bool cur_exact = true;
    EstState est{0u, 0u, {0.0f, 0.0f}};  // (the launch starts with exact terms)
    CostIv cur_iv{cur_total, cur_total};
    typename RngOf<XW, L>::type rng;
    rng_load(rng, a, chain, m0);
    uint64_t accepted = m0.accepted;
    float best_total = m0.best_total;
    double beta = kBeta;
    if constexpr (TRACK)  // (the extended variants also carry parallel tempering)
        if (a.n_temps > 1) beta = a.ladder[m0.rung];
#if MH_STAMPS
    unsigned long long cyc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_last;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_last) :: "memory");
#endif
#if MH_CHECK
    float chk_cur = cur_total;  // (check builds: the current total, always exact)
#endif

#pragma clang loop unroll(disable)
    for (int it = 0; it < a.iterations; ++it) {
        for (int w = r; w < ch.SW; w += L) stage(ch.SAMB).put(w, ch.SAM[w]);
        rng_prepare(rng);
        const int2 kk = propose<S>(rng, *rm_l, frozen, ch, o, r, writer);
        const int ka = kk.x, kb = kk.y;
        // the proposal's poses and boxes, its undo record, the SurfaceArea bits' backup
        hand_off(ch.X, ch.Y, ch.BOX, ch.RYF, ch.aux, ch.SAMB);
        // Objects ka (lane 0) and kb (lane 1): FocalPoint term, SurfaceArea bits, wildness.
        int dwild = 0;
        const double rka = obj_ry<S>(o, ka < 0 ? 0 : ka), rkb = obj_ry<S>(o, kb < 0 ? 0 : kb);
        float sv_obj = 0.0f, sv_clr = 0.0f;  // (lanes 0, 1: the moved objects' SurfaceArea sums)
        EstState est_bk = est;  // (the undo's record, undo_proposal)
        bool kest = false;      // (lanes 0, 1: their object's FocalPoint term is an estimate)
        if (r < 2) {
            const int k = r == 0 ? ka : kb;
            if (k >= 0) {
                const ObjP p = obj_pose(ch, k);
                // the plain step's FocalPoint estimate (exact where cph_est cannot vouch for it)
                bool ambo = true;
                float w = 0.0f;
                if constexpr (!TRACK) {
                    const float fy = rm_l->fyf - p.yf, fx = rm_l->fxf - p.xf;
                    ambo = !(fmaxf(fabsf(fy), fabsf(fx)) >= 0x1p-100f);
                    w = cph_est(atan2_est(fy, fx), p, ambo);
                }
                if (ambo) w = focal_cos(*rm_l, p.xf, p.yf, p.rotYf);
                stage(ch.CPH).put(k, -w);
                kest = !ambo;
                const float4 vo = comp_overlaps(*rm_l, ch.BOX[k]);
                sam_put(ch, c + k, nonzero4(vo));
                sv_obj = nonzero4(vo) ? (vo.x + vo.y) + (vo.z + vo.w) : 0.0f;
                if (k < c) {
                    const float4 vc = comp_overlaps(*rm_l, shape_box(ch.clrs[k], p.xf, p.yf));
                    sam_put(ch, k, nonzero4(vc));
                    sv_clr = nonzero4(vc) ? (vc.x + vc.y) + (vc.z + vc.w) : 0.0f;
                }
                const DBackup& ob = ch.aux->b[r];
                dwild = (wild_pose(ch.X[k], ch.Y[k], r == 0 ? rka : rkb) ? 1 : 0) -
                        (wild_pose(ob.x, ob.y, ob.ry) ? 1 : 0);
            }
        }
        const int wild_star = wild_cnt + __shfl(dwild, 0) + __shfl(dwild, 1);
        if constexpr (!TRACK) {  // the moved objects' owner lanes record the estimates
            const bool ea = __builtin_amdgcn_readlane((int)kest, 0) != 0;
            const bool eb = __builtin_amdgcn_readlane((int)kest, 1) != 0;
            if (ka >= 0 && r == (ka & 63))
                est.obj = ea ? (est.obj | (1u << (ka >> 6))) : (est.obj & ~(1u << (ka >> 6)));
            if (kb >= 0 && r == (kb & 63))
                est.obj = eb ? (est.obj | (1u << (kb >> 6))) : (est.obj & ~(1u << (kb >> 6)));
        }
        hand_off(ch.CPH, ch.SAM);  // the moved objects' FocalPoint terms and SurfaceArea bits
        DSTAMP(0);
        typename Own<S>::wvec bk_nz = o.nz0;  // (the undo's record, undo_proposal)
        const bool chg0 = clearance_delta<S>(ch, o, n, c, ka, kb, r);
        DSTAMP(1);
        RelBk rbk;
        rels_delta(ch, nr, ka, kb, r, &rbk, TRACK ? nullptr : &est);
        DSTAMP(2);
        symmetry_delta<S>(ch, o, n, ka, kb, wild_star > 0, r);
        hand_off(ch.CLA, ch.NZ, ch.RPW, ch.RANG);  // the proposal's pairs and relationship terms
        DSTAMP(3);
        // Plain chains: Accept's uniform (the next draw after the proposal's, Kernel.cu:710) is
        // drawn first. The Clearance and SurfaceArea lists are built with the bound's partial
        // sums, and a proposal the bound already rejects skips the replay.
        constexpr bool FASTD = !TRACK;
        int bd = BOUND_OPEN;
        CostIv star_iv{0.0f, 0.0f};
        float u_acc = 0.0f;
        float clsum = 0.0f, sasum = 0.0f, clpos = 0.0f;
        int kcl = 0, cnt_cl = 0;
        bool cl_built = false;  // (the Clearance list for the replay is written)
        ClRow rc_star = rc_cur;  // the proposal's first-row Clearance sums
        if (FASTD && c <= 64) {
            const ClRow f = cl_row0<S>(ch, o, c, r, chg0);
            if (chg0) rc_star = f;
            const int cnt = r < c ? rc_star.cnt : 0;
            const int base0 = group_excl_scan<L>(cnt, r, cnt_cl);
            if (r < c) {
                clsum = rc_star.sum;
                kcl = cnt;
                clpos = fmaf((float)base0, -rc_star.sum, rc_star.pos);
            }
        } else {
            cnt_cl = build_cl_list<S>(ch, o, c, r, 0, &clsum, &kcl, &clpos);
            cl_built = true;
        }
#if MH_CHECK
        if (!cl_built) {  // the cached row sums against a fresh build
            float cs = 0.0f, cp = 0.0f;
            int kc = 0;
            const int cn = build_cl_list<S>(ch, o, c, r, 0, &cs, &kc, &cp);
            MH_CK(cs == clsum && kc == kcl && cn == cnt_cl &&
                      fabsf(cp - clpos) <= 1e-5f * fabsf(cp) + 1e-30f,
                  27, __float_as_uint(cs), __float_as_uint(clsum));
            cl_built = true;
        }
#endif
        // SurfaceArea: the cached entry sums with the moved objects' entries replaced (lanes 0 and
        // 1 computed them above); the list itself only for the steps that replay
        const float sv[4] = {__shfl(sv_obj, 0), __shfl(sv_clr, 0), __shfl(sv_obj, 1),
                             __shfl(sv_clr, 1)};
        const int se[4] = {ka >= 0 ? c + ka : -1, ka >= 0 && ka < c ? ka : -1,
                           kb >= 0 ? c + kb : -1, kb >= 0 && kb < c ? kb : -1};
        int cnt_sa = 0;
        bool sa_built = false;
        if constexpr (FASTD) {
#pragma unroll
            for (int t = 0; t < 2 * S; ++t) {
                const int e = t * L + r;
                float v = o.sav[t];
#pragma unroll
                for (int q = 0; q < 4; ++q) v = e == se[q] ? sv[q] : v;
                sasum -= v;
            }
        } else {
            cnt_sa = build_sa_list(ch, n, c, r, 0, &sasum);
            sa_built = true;
        }
#if MH_CHECK
        if (!sa_built) {  // the cached entry sums against a fresh build
            float sf = 0.0f;
            cnt_sa = build_sa_list(ch, n, c, r, 0, &sf);
            MH_CK(sf == sasum, 29, __float_as_uint(sf), __float_as_uint(sasum));
            sa_built = true;
        }
#endif
        if constexpr (FASTD) {
            u_acc = rng.uniform();
            BoundTerms bt = delta_bound_terms<S>(ch, o, n, c, nr, r, est);
            bt.cl = clsum;
            bt.kcl = kcl;
            bt.clpos = clpos;
            bt.sa = sasum;
            // (not on a launch's last step: it ends with the current costs exact, through the
            // exact pass below when they are not)
            if (it + 1 < a.iterations)
                bd = bound_decide<true>(*rm_l, n, c, nr, cnt_cl, bt, u_acc, cur_iv, star_iv,
                                        a.bound_slack);
        }
#if MH_STAMPS > 1
        if (r == 0) {
            atomicAdd(&g_delta_counts[4], 1ull);
            atomicAdd(&g_delta_counts[5], (unsigned long long)(bd == BOUND_REJECT ? 1 : 0));
            atomicAdd(&g_delta_counts[6], (unsigned long long)(bd == BOUND_ACCEPT ? 1 : 0));
        }
#endif
#if MH_CHECK
        if (FASTD && r == 0) mh_count_decision(bd, it + 1 < a.iterations);
        // Check builds verify every decision the bound takes against the exact costs (the
        // replay of the lists just built): the proposal's exact total lies in the bound's
        // interval, the current total in the carried one, a certain REJECT / ACCEPT is Accept's.
        float chk_star = 0.0f;
        if (FASTD && bd != BOUND_OPEN) {
            float ro[8];
            fix_estimates<S>(ch, o, est, r);  // (the check's replay needs the exact terms)
            replay_config<S>(ch, o.pmx, o, n, cnt_cl, cnt_sa, r, ro);
            chk_star = uniform_f(ro[0]);
            const bool acc_x = u_acc < accept_threshold(kBeta * ((double)chk_star - (double)chk_cur));
            if (r == 0) {
                atomicAdd(&g_check[5], 1u);
                MH_CK(chk_star >= star_iv.lo && chk_star <= star_iv.hi, 22,
                      __float_as_uint(chk_star), __float_as_uint(star_iv.hi - star_iv.lo));
                MH_CK(bd != BOUND_REJECT || !acc_x, 20, __float_as_uint(chk_star),
                      __float_as_uint(chk_cur));
                MH_CK(bd != BOUND_ACCEPT || acc_x, 21, __float_as_uint(chk_star),
                      __float_as_uint(chk_cur));
            }
        }
        if (FASTD && r == 0)
            MH_CK(chk_cur >= cur_iv.lo && chk_cur <= cur_iv.hi, 23, __float_as_uint(chk_cur),
                  __float_as_uint(cur_iv.hi - cur_iv.lo));
#endif
        float sc[8];
        bool rare = false;  // the exact pass of the current configuration ran (below)
        int bd2 = BOUND_OPEN;  // an open step decided by its exact total against the interval
        if (bd == BOUND_OPEN) {
        if constexpr (!TRACK) fix_estimates<S>(ch, o, est, r);  // (the replay reads exact terms)
        if (!cl_built) build_cl_list<S>(ch, o, c, r, 0);  // (the lists the replay walks)
        if (!sa_built) cnt_sa = build_sa_list(ch, n, c, r, 0);
#if MH_STAMPS > 1
        if (r == 0) {
            atomicAdd(&g_delta_counts[0], (unsigned long long)cnt_cl);
            atomicAdd(&g_delta_counts[1], (unsigned long long)cnt_sa);
            atomicAdd(&g_delta_counts[2], (unsigned long long)(cnt_cl > ch.cap_cl));
            atomicAdd(&g_delta_counts[3], (unsigned long long)(cnt_sa > ch.cap_sa));
        }
#endif
        DSTAMP(4);
        // Pass 0 replays the proposal's sums. When the current total is only an interval
        // (FASTD, cur_exact false), pass 1 undoes the proposal and replays the current
        // configuration's sums; one replay call site, so the rare pass adds no registers.
        int lcl = cnt_cl, lsa = cnt_sa;
#pragma clang loop unroll(disable)
        for (int pass = 0;; ++pass) {
            float ro[8];
            typename Own<S>::fvec mx = o.pmx;
            if (pass) mx = o.cmx;
#if MH_STAMPS
            replay_config<S>(ch, mx, o, n, lcl, lsa, r, ro, &cyc[7]);
#else
            replay_config<S>(ch, mx, o, n, lcl, lsa, r, ro);
#endif
            if (pass) {
#pragma unroll
                for (int k = 0; k < 8; ++k) cur[k] = uniform_f(ro[k]);
                cur_total = cur[0];
#if MH_CHECK
                if (r == 0) {
                    MH_CK(cur_total == chk_cur, 24, __float_as_uint(cur_total),
                          __float_as_uint(chk_cur));
                    atomicAdd(&g_decide[3], 1ull);
                }
#endif
                cur_exact = true;
                cur_iv = CostIv{cur_total, cur_total};
                break;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) sc[k] = uniform_f(ro[k]);  // (scalar registers)
            if (!FASTD || cur_exact) break;
            // The proposal's exact total often decides against the current total's interval
            // alone (decide_exact_star): then no exact pass of the current configuration. (Not
            // on a launch's last step: a rejection would leave the current costs inexact, and a
            // launch ends with them exact.)
            if (it + 1 < a.iterations) bd2 = decide_exact_star(sc[0], cur_iv, u_acc, kBeta);
#if MH_CHECK
            if (r == 0 && bd2 != BOUND_OPEN) {
                const bool acc_x = u_acc < accept_threshold(kBeta * ((double)sc[0] - (double)chk_cur));
                MH_CK(acc_x == (bd2 == BOUND_ACCEPT), 25, __float_as_uint(sc[0]),
                      __float_as_uint(chk_cur));
            }
#endif
            if (bd2 != BOUND_OPEN) break;
            // The decision needs the current configuration's exact costs: undo the proposal.
            // The undo records are swapped to its objects' poses and FocalPoint terms (and SAMB
            // keeps its SurfaceArea bits), so a second undo_proposal() re-applies it.
            const int nb = ch.aux->nb;
            const DBackup p0 = read_obj<S>(ch, o, nb > 0 ? ch.aux->b[0].k : 0);
            const DBackup p1 = read_obj<S>(ch, o, nb > 1 ? ch.aux->b[1].k : 0);
            undo_proposal<S>(ch, o, n, c, nr, ka, kb, r, writer, rbk, bk_nz, est, est_bk);
            if (writer) {
                if (nb > 0) stage(ch.aux)->b[0] = p0;
                if (nb > 1) stage(ch.aux)->b[1] = p1;
            }
            if constexpr (!TRACK) fix_estimates<S>(ch, o, est, r);  // (the current configuration's)
            lcl = build_cl_list<S>(ch, o, c, r, 0);
            lsa = build_sa_list(ch, n, c, r, 0);
            rare = true;
#if MH_STAMPS > 1
            if (r == 0) atomicAdd(&g_delta_counts[7], 1ull);
#endif
        }
        DSTAMP(5);
        } else {
        DSTAMP(4);
        }
        // Best-of-chain: star is judged before Accept, Kernel.cu:808-816.
        if constexpr (TRACK) {
            if (a.track != TRACK_OFF && best_improves(a.track, sc[0], best_total)) {
                best_total = sc[0];
                save_best_delta<S>(ch, o, a.best + chain * (int64_t)(F_COUNT * n), n, r);
            }
        }
        bool acc;
        if constexpr (TRACK) acc = accept_at(rng, sc[0], cur_total, beta);
        else if (bd != BOUND_OPEN) acc = bd == BOUND_ACCEPT;
        else if (bd2 != BOUND_OPEN) acc = bd2 == BOUND_ACCEPT;
        else acc = u_acc < accept_threshold(kBeta * ((double)sc[0] - (double)cur_total));
        // A rejected proposal is undone; after the exact pass of the current configuration
        // (rare) the state is the current one, and an accepted proposal is re-applied.
        if (acc == rare) undo_proposal<S>(ch, o, n, c, nr, ka, kb, r, writer, rbk, bk_nz, est, est_bk);
        if (acc) {
            ++accepted;
#if MH_CHECK
            chk_cur = bd == BOUND_OPEN ? sc[0] : chk_star;
#endif
            rc_cur = rc_star;
#pragma unroll
            for (int t = 0; t < 2 * S; ++t) {  // (the proposal's SurfaceArea entry sums)
                const int e = t * L + r;
#pragma unroll
                for (int q = 0; q < 4; ++q) o.sav[t] = e == se[q] ? sv[q] : o.sav[t];
            }
            o.cmx = o.pmx;
            o.carg = o.parg;
            wild_cnt = wild_star;
            if (FASTD && bd == BOUND_ACCEPT) {
                cur_exact = false;
                cur_iv = star_iv;
            } else {
                cur_total = sc[0];
                if constexpr (FASTD) {
                    cur_exact = true;
                    cur_iv = CostIv{cur_total, cur_total};
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) cur[k] = uniform_f(sc[k]);
            }
            if (writer) commit_swap_zrr(ch, n);
            hand_off(ch.aux);  // (the step's undo record is read no more)
        }
        DSTAMP(6);
    }
#if MH_STAMPS
    if (r == 0)
        for (int k = 0; k < 8; ++k) atomicAdd(&g_delta_cycles[k], cyc[k]);
#endif

#if MH_CHECK
    if (!TRACK && r == 0)  // a launch ends with the current configuration's exact costs
        MH_CK(cur[0] == chk_cur, 26, __float_as_uint(cur[0]), __float_as_uint(chk_cur));
#endif
    if (writer) {
        ChainMeta m;
        m.draws = rng.draws;
        m.accepted = accepted;
        m.bm_has = rng.bm_has;
        m.bm_val = rng.bm_val;
        rng_save(rng, a, chain);
        for (int k = 0; k < 8; ++k) m.costs[k] = cur[k];
        m.best_total = best_total;
        m.rung = m0.rung;
        a.meta[chain] = m;
    }
    double* dst = a.st + chain * (int64_t)(F_COUNT * n);
#pragma unroll
    for (int t = 0; t < S; ++t) {
        const int i = t * L + r;
        if (i < n) {
            dst[F_X * n + i] = ch.X[i];
            dst[F_Y * n + i] = ch.Y[i];
            dst[F_RY * n + i] = o.ry[t];
        }
    }
}

template <int S>
hipError_t launch_delta_s(const LaunchArgs& a, int waves_per_wg, hipStream_t stream) {
    const int64_t blocks = (a.n_chains + waves_per_wg - 1) / waves_per_wg;
    const size_t lds = (size_t)a.dlay.hdr + (size_t)waves_per_wg * a.dlay.stride;
    const dim3 grid((unsigned)blocks), block((unsigned)(64 * waves_per_wg));
    if (a.rng == RNG_CURAND_XORWOW)  // (tracking compiled in, switched at run time)
        hipLaunchKernelGGL((mh_delta_kernel<S, true, true>), grid, block, lds, stream, a);
    else if (a.track != TRACK_OFF || a.n_temps > 1)
        hipLaunchKernelGGL((mh_delta_kernel<S, false, true>), grid, block, lds, stream, a);
    else
        hipLaunchKernelGGL((mh_delta_kernel<S, false, false>), grid, block, lds, stream, a);
    return hipGetLastError();
}

}  // namespace

#if MH_CHECK
extern "C" __attribute__((visibility("default"))) int mh_debug_check_delta(unsigned int* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_check), sizeof(unsigned int) * 8) == hipSuccess ? 0 : -1;
}
extern "C" __attribute__((visibility("default"))) int mh_debug_decisions_delta(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_decide), sizeof(unsigned long long) * 4) ==
                   hipSuccess ? 0 : -1;
}
#endif

#if MH_STAMPS
extern "C" __attribute__((visibility("default"))) int mh_debug_delta_cycles(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_delta_cycles), sizeof(unsigned long long) * 8) !=
        hipSuccess)
        return -1;
    return hipMemcpyFromSymbol(out + 8, HIP_SYMBOL(g_delta_counts), sizeof(unsigned long long) * 8) ==
                   hipSuccess ? 0 : -1;
}
#endif

// Object slots per lane of the instance that serves n objects.
static int delta_slots(int n) { return n <= 64 ? 1 : n <= 128 ? 2 : n <= 256 ? 4 : 8; }
int delta_max_waves(int n) { return delta_max_waves_s(delta_slots(n)); }

size_t delta_lds_bytes(const DeltaLds& lay, int waves_per_wg) {
    return (size_t)lay.hdr + (size_t)waves_per_wg * lay.stride;
}

// Resident workgroups per CU of the plain step kernel for n objects and a workgroup of
// `waves_per_wg` chains (registers, LDS and the wave limit all counted by the runtime). 0 if it
// does not fit.
int delta_blocks_per_cu(int n, int waves_per_wg, size_t lds_bytes) {
    int blocks = 0;
    hipError_t e = hipErrorInvalidValue;
    const int threads = 64 * waves_per_wg;
    switch (delta_slots(n)) {
        case 1: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_delta_kernel<1, false, false>, threads, lds_bytes); break;
        case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_delta_kernel<2, false, false>, threads, lds_bytes); break;
        case 4: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_delta_kernel<4, false, false>, threads, lds_bytes); break;
        default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_delta_kernel<8, false, false>, threads, lds_bytes); break;
    }
    return e == hipSuccess ? blocks : 0;
}

hipError_t launch_delta(const LaunchArgs& a, int waves_per_wg, hipStream_t s) {
    if (a.n_chains <= 0) return hipSuccess;
    switch (delta_slots(a.rm.n)) {
        case 1: return launch_delta_s<1>(a, waves_per_wg, s);
        case 2: return launch_delta_s<2>(a, waves_per_wg, s);
        case 4: return launch_delta_s<4>(a, waves_per_wg, s);
        default: return launch_delta_s<8>(a, waves_per_wg, s);
    }
}

}  // namespace mh
