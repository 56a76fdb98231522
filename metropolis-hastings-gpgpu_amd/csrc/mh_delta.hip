// mh_delta.hip -- the MH step (Kernel.cu:785-828) with incremental cost evaluation.
//
// A proposal changes at most two objects (propose(), Kernel.cu:576-704), so almost every term
// of Costs() (Kernel.cu:516-550) is the same before and after it. This kernel keeps, per chain
// and in LDS, every quantity a proposal can only change locally, recomputes just the affected
// entries, and replays the reference's ordered float/double sums from the cached terms:
//   * FocalPoint: -cos(phi_i) per object (the .w word of the pose record);
//   * Symmetry: each row's exact maximum and its argmax, double-buffered (current / proposed);
//     a proposal re-scans the changed rows and folds the changed columns into the others;
//   * Clearance: the non-zero (clearance, object) overlap pairs as a bit matrix, updated by
//     row (clearances whose source moved) and by column (moved objects);
//   * SurfaceArea: a bit per non-zero entry;
//   * PairWise / PairWiseAngle: the term of every relationship, recomputed when one of its
//     objects moved;
//   * VisualBalance needs no cache (area * x is one product).
// The values that enter every sum are the reference's own (same functions as the full
// evaluation, mh_common.h); only the work to find them changes, so costs -- and chains -- stay
// bit-identical to the oracle. Unlike the full evaluation (mh_chain.hip), where one 64-lane
// wavefront serves one chain, the per-step work here is small and a wavefront carries 64/L
// chains (L = 8..32 lanes each); lane k < 8 of a chain replays ordered sum k.

#include <stdint.h>
#include <stdlib.h>

#include "mh_common.h"

#ifndef MH_STAMPS
#define MH_STAMPS 0  // diagnostic builds: cycles per phase of the step (tools/stamps.py --delta)
#endif
#if MH_STAMPS
__device__ unsigned long long g_delta_cycles[8];
__device__ unsigned long long g_delta_counts[4];  // sum of Clearance / SurfaceArea list sizes, overflows
#define DSTAMP(k) do { __builtin_amdgcn_sched_barrier(0); unsigned long long _t; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t) :: "memory"); cyc[k] += _t - t_last; t_last = _t; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define DSTAMP(k) do { } while (0)
#endif

namespace mh {
namespace {

struct RowMax {  // one symmetry row: exact max(0, max_j value) and the j attaining it (-1: 0)
    float mx;
    int arg;
};

// Symmetry rows of one buffer: -(row max) (the replay's term) and the argmax.
struct RowBuf {
    float* nmx;
    int* arg;
    __device__ __forceinline__ RowMax get(int i) const { return RowMax{-nmx[i], arg[i]}; }
    __device__ __forceinline__ void put(int i, RowMax v) const {
        nmx[i] = -v.mx;
        arg[i] = v.arg;
    }
};

struct DBackup {  // an object's cost-relevant pose and FocalPoint term before a proposal
    int k;
    float w;
    double x, y, ry;
};

struct DeltaAux {
    DBackup b[2];
    int nb;
    int swap_a, swap_b;
    int pad0;
    float cur[8];  // resultCosts of the current configuration
};
static_assert(sizeof(DeltaAux) <= 192, "DeltaAux");

struct DeltaPtrs {
    const ObjConst* objc;
    const ClrConst* clrc;
    const RelConst* relc;
    const DevRoom* rm;
    const float *AREA, *ONES;  // replay streams shared by the workgroup
    const double* ZERO;
    double *X, *Y, *RY;
    ObjP* P;
    float* CPH;   // -cos(phi_i)
    RowBuf RB[2];
    float4* CLA;
    uint64_t* NZ;
    uint32_t *SAM, *SAMB;
    double *RPW, *RANG;
    float *LCL, *LSA;
    DeltaAux* aux;
    double* zrr;  // HBM: z, rotX, rotZ rows of this chain
    int W, SW, cap_cl, cap_sa, NP, NR, DL;
};

// ---- per-object quantities --------------------------------------------------------------------

__device__ __forceinline__ float4 obj_box(const DeltaPtrs& ch, int j) {
    const ObjP p = ch.P[j];
    return shape_box(ch.objc[j].off, p.xf, p.yf);
}

__device__ __forceinline__ float4 cla_box(const DeltaPtrs& ch, int ci) {
    const ClrConst& cc = ch.clrc[ci];
    const ObjP p = ch.P[cc.src];
    return shape_box(cc.shape, p.xf, p.yf);
}

// SurfaceAreaCosts entry e (Kernel.cu:453-480): clearance e's box at cfg[e] (the reference's
// quirk, :456) for e < C, then object e - C's off-limits box.
__device__ __forceinline__ float4 sa_entry(const DeltaPtrs& ch, int c, int e) {
    if (e < c) {
        const ObjP p = ch.P[e];
        return comp_overlaps(*ch.rm, shape_box(ch.clrc[e].shape, p.xf, p.yf));
    }
    return comp_overlaps(*ch.rm, obj_box(ch, e - c));
}

// FocalPointCosts term of object i, Kernel.cu:271,277 with phi() of :185-188.
__device__ __forceinline__ float focal_cos(const DevRoom& rm, ObjP p) {
    const float at = atan2_f32(rm.fyf - p.yf, rm.fxf - p.xf);
    const float b = at - p.rotYf;
    const float ph = (float)((double)b + kHalfPI);
    return cos_f32(ph);
}

// SymmetryCosts row setup of object i, Kernel.cu:292-299.
__device__ __forceinline__ void row_setup(const DeltaPtrs& ch, int i, float& rx, float& ry,
                                          float& rr) {
    const DevRoom& rm = *ch.rm;
    const double x = ch.X[i], y = ch.Y[i], ryi = ch.RY[i];
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
    if (nz) atomicOr(&ch.SAM[e >> 5], bit);
    else atomicAnd(&ch.SAM[e >> 5], ~bit);
}

// ---- symmetry rows ------------------------------------------------------------------------

// Exact row maximum of row i over every column, the group's lanes sharing the columns: fp32
// estimates screen the pairs (sym_err bounds their error), the leader is evaluated exactly and
// an ambiguous top two falls back to the exact value of every candidate within the bound.
template <int L>
__device__ RowMax scan_row(const DeltaPtrs& ch, int n, int i, bool exact_mode, int r, int gbase) {
    float rx, ry, rr;
    row_setup(ch, i, rx, ry, rr);
    float t1 = -INFINITY, t2 = -INFINITY;
    int tj = -1;
    for (int j = r; j < n; j += L) {
        const float v = sym_val_fast(*reinterpret_cast<const float4*>(&ch.P[j]), rx, ry, rr);
        t2 = __builtin_amdgcn_fmed3f(t1, t2, v);
        const bool up = v > t1;
        t1 = up ? v : t1;
        tj = up ? j : tj;
    }
    const SymLead ld = group_sym_lead<L>(t1, t2, tj, r, gbase, rr);
    RowMax out;
    if (!exact_mode && ld.clear) {
        const ObjP q = ch.P[ld.j];
        const float e = sym_val_exact(q.xf, q.yf, ch.RY[ld.j], rx, ry, (double)rr);
        out.mx = fmaxf(0.0f, e);
        out.arg = e > 0.0f ? ld.j : -1;
        return out;
    }
    const float thr =
        (exact_mode || ld.j < 0) ? INFINITY : 2.0f * sym_err(fabsf(ld.m) + 1.0f, rr);
    float bv = -INFINITY;
    int bj = -1;
    for (int j = r; j < n; j += L) {
        const ObjP p = ch.P[j];
        const float v = sym_val_fast(*reinterpret_cast<const float4*>(&p), rx, ry, rr);
        if (!(v < ld.m - thr)) {
            const float e = sym_val_exact(p.xf, p.yf, ch.RY[j], rx, ry, (double)rr);
            if (e > bv) {
                bv = e;
                bj = j;
            }
        }
    }
    group_max_arg<L>(bv, bj);
    out.mx = bv > 0.0f ? bv : 0.0f;
    out.arg = bv > 0.0f ? bj : -1;
    return out;
}

// Rows of the configuration in LDS after objects ka, kb (-1: none) changed, from the rows of the
// configuration before (cur) into nxt. Lane r owns rows r, r + L, ...
template <int L>
__device__ void symmetry_delta(const DeltaPtrs& ch, int n, const RowBuf cur, const RowBuf nxt,
                               int ka, int kb, bool exact_mode, int r, int gbase) {
    float4 qa = make_float4(0.f, 0.f, 0.f, 0.f), qb = qa;
    if (ka >= 0) qa = *reinterpret_cast<const float4*>(&ch.P[ka]);
    if (kb >= 0) qb = *reinterpret_cast<const float4*>(&ch.P[kb]);
    uint64_t pa = 0, pb = 0, resc = 0;
    int t = 0;
    for (int i = r; i < n; i += L, ++t) {
        const RowMax c0 = cur.get(i);
        nxt.put(i, c0);
        if (i == ka || i == kb) {
            resc |= 1ull << t;
            continue;
        }
        float rx, ry, rr;
        row_setup(ch, i, rx, ry, rr);
        // pending unless certainly below the old maximum; a maximum held by the changed
        // column that certainly dropped sends the row straight to the re-scan
        if (ka >= 0) {
            const float v = sym_val_fast(qa, rx, ry, rr);
            const bool below = !exact_mode && v + sym_err(v, rr) < c0.mx;
            if (c0.arg == ka && below) resc |= 1ull << t;
            else if (!below) pa |= 1ull << t;
        }
        if (kb >= 0) {
            const float v = sym_val_fast(qb, rx, ry, rr);
            const bool below = !exact_mode && v + sym_err(v, rr) < c0.mx;
            if (c0.arg == kb && below) resc |= 1ull << t;
            else if (!below) pb |= 1ull << t;
        }
    }
    pa &= ~resc;
    pb &= ~resc;
    // Exact values of the pending (row, column) pairs, one per lane per pass.
    while (__ballot((pa | pb) != 0)) {
        if (pa | pb) {
            int tt, col;
            if (pa) {
                tt = __builtin_ctzll(pa);
                pa &= pa - 1;
                col = ka;
            } else {
                tt = __builtin_ctzll(pb);
                pb &= pb - 1;
                col = kb;
            }
            const int i = tt * L + r;
            float rx, ry, rr;
            row_setup(ch, i, rx, ry, rr);
            const ObjP q = ch.P[col];
            const float e = sym_val_exact(q.xf, q.yf, ch.RY[col], rx, ry, (double)rr);
            const RowMax c0 = cur.get(i);
            const RowMax s0 = nxt.get(i);
            if (col == c0.arg && !(e >= c0.mx)) {
                resc |= 1ull << tt;  // the old maximum is gone: re-scan the row
            } else if (e > s0.mx) {
                nxt.put(i, RowMax{e, col});
            }
        }
    }
    // Re-scans, one row per chain at a time across the chain's lanes.
    for (;;) {
        const uint64_t who = group_ballot<L>(resc != 0, gbase);
        if (who == 0) break;
        const int b = __builtin_ctzll(who);
        const int tb = __shfl(resc ? __builtin_ctzll(resc) : 0, gbase + b);
        const int i = tb * L + b;
        const RowMax s = scan_row<L>(ch, n, i, exact_mode, r, gbase);
        if (r == b) {
            nxt.put(i, s);
            resc &= resc - 1;
        }
    }
}

// ---- clearance pairs ------------------------------------------------------------------------

// Row ci of the non-zero bit matrix from scratch (the group's lanes share the objects).
template <int L>
__device__ void nz_row(const DeltaPtrs& ch, int n, int ci, int r, int gbase) {
    const float4 A = ch.CLA[ci];
    for (int w = 0; w < ch.W; ++w) {
        uint64_t word = 0;
#pragma unroll
        for (int qq = 0; qq < 64 / L; ++qq) {
            const int j = w * 64 + qq * L + r;
            const bool nz = j < n && overlap(A, obj_box(ch, j)) != 0.0f;
            const uint64_t bits = group_ballot<L>(nz, gbase);
            word |= (L == 64) ? bits : (bits << (qq * L));
        }
        if (r == 0) ch.NZ[ci * ch.W + w] = word;
    }
}

// Clearance boxes and pair bits after objects ka, kb changed (also restores them after a
// rejected proposal has put the old poses back).
template <int L>
__device__ void clearance_delta(const DeltaPtrs& ch, int n, int c, int ka, int kb, int r,
                                int gbase) {
    if (ka < 0 && kb < 0) return;
    uint64_t rows = 0;
    int t = 0;
    for (int ci = r; ci < c; ci += L, ++t) {
        const int src = ch.clrc[ci].src;
        if (src == ka || src == kb) {
            ch.CLA[ci] = cla_box(ch, ci);
            rows |= 1ull << t;
        }
    }
    wave_sync();
    // Columns ka, kb of the rows whose clearance did not move (lane-owned rows).
    for (int s = 0; s < 2; ++s) {
        const int j = s == 0 ? ka : kb;
        if (j < 0) continue;
        const float4 bj = obj_box(ch, j);
        const uint64_t bit = 1ull << (j & 63);
        t = 0;
        for (int ci = r; ci < c; ci += L, ++t) {
            if (rows & (1ull << t)) continue;
            uint64_t* wd = &ch.NZ[ci * ch.W + (j >> 6)];
            const bool nz = overlap(ch.CLA[ci], bj) != 0.0f;
            *wd = nz ? (*wd | bit) : (*wd & ~bit);
        }
    }
    // Rows of the clearances that moved, one per chain at a time.
    for (;;) {
        const uint64_t who = group_ballot<L>(rows != 0, gbase);
        if (who == 0) break;
        const int b = __builtin_ctzll(who);
        const int tb = __shfl(rows ? __builtin_ctzll(rows) : 0, gbase + b);
        nz_row<L>(ch, n, tb * L + b, r, gbase);
        if (r == b) rows &= rows - 1;
    }
}

// PairWise / PairWiseAngle terms of the relationships touching ka or kb (or all, ka = -2).
template <int L>
__device__ void rels_delta(const DeltaPtrs& ch, int nr, int ka, int kb, int r) {
    uint64_t pend = 0;
    int t = 0;
    for (int q = r; q < nr; q += L, ++t) {
        const RelConst& rc = ch.relc[q];
        const bool hit = ka == -2 || rc.s == ka || rc.t == ka || rc.as == ka || rc.at == ka ||
                         (kb >= 0 && (rc.s == kb || rc.t == kb || rc.as == kb || rc.at == kb));
        if (hit) pend |= 1ull << t;
    }
    while (__ballot(pend != 0)) {
        if (pend) {
            const int q = __builtin_ctzll(pend) * L + r;
            pend &= pend - 1;
            double tpw, tang;
            rel_terms(ch.relc[q], ch.P, tpw, tang);
            ch.RPW[q] = -tpw;
            ch.RANG[q] = -tang;
        }
    }
}

// ---- compacted Clearance / SurfaceArea terms ------------------------------------------------

// Non-zero Clearance terms, clearance-major then object (Kernel.cu:408-431), negated: those at
// positions [lo, lo + cap_cl) go to LCL[pos - lo]. Returns the total count.
template <int L>
__device__ int build_cl_list(const DeltaPtrs& ch, int c, int r, int lo) {
    int base = 0;
    for (int cb = 0; cb < c; cb += L) {
        const int ci = cb + r;
        int cnt = 0;
        if (ci < c)
            for (int w = 0; w < ch.W; ++w) cnt += __builtin_popcountll(ch.NZ[ci * ch.W + w]);
        int tot;
        int pos = base + group_excl_scan<L>(cnt, r, tot);
        if (cnt) {
            const float4 A = ch.CLA[ci];
            for (int w = 0; w < ch.W; ++w) {
                uint64_t word = ch.NZ[ci * ch.W + w];
                while (word) {
                    const int j = w * 64 + __builtin_ctzll(word);
                    word &= word - 1;
                    if (pos >= lo && pos < lo + ch.cap_cl)
                        ch.LCL[pos - lo] = -overlap(A, obj_box(ch, j));
                    ++pos;
                }
            }
        }
        base += tot;
    }
    return base;
}

// Non-zero SurfaceArea terms in the reference's order, negated: positions [lo, lo + cap_sa) go
// to LSA[pos - lo]. Returns the total count.
template <int L>
__device__ int build_sa_list(const DeltaPtrs& ch, int n, int c, int r, int lo) {
    int base = 0;
    const int ne = c + n;
    for (int eb = 0; eb < ne; eb += L) {
        const int e = eb + r;
        const bool set = e < ne && ((ch.SAM[e >> 5] >> (e & 31)) & 1u);
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        int cnt = 0;
        if (set) {
            v = sa_entry(ch, c, e);
            cnt = (v.x != 0.0f) + (v.y != 0.0f) + (v.z != 0.0f) + (v.w != 0.0f);
        }
        int tot;
        int pos = base + group_excl_scan<L>(cnt, r, tot);
        if (cnt) {
            const float tv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (tv[u] != 0.0f) {
                    if (pos >= lo && pos < lo + ch.cap_sa) ch.LSA[pos - lo] = -tv[u];
                    ++pos;
                }
        }
        base += tot;
    }
    return base;
}

// ---- terms for the rejection bound (certain_reject, mh_common.h) --------------------------

// This lane's partial sums of every term of Costs() for the configuration in LDS: its objects
// (VisualBalance, FocalPoint, Symmetry rows in `nmx`), its relationships, its clearances' non-zero
// pairs and its SurfaceArea entries. `ncl` returns the chain's count of non-zero Clearance terms.
template <int L>
__device__ BoundTerms delta_bound_terms(const DeltaPtrs& ch, int n, int c, int nr,
                                        const float* nmx, int r, int& ncl) {
    BoundTerms bt;
    bt.nx = bt.ny = bt.anx = bt.any = bt.fp = bt.afp = bt.sym = bt.cl = bt.sa = 0.0f;
    bt.pw = bt.ang = bt.aang = 0.0f;
    for (int i = r; i < n; i += L) {
        const float a = ch.AREA[i];
        const float tx = (float)((double)a * ch.X[i]), ty = (float)((double)a * ch.Y[i]);
        bt.nx += tx;
        bt.ny += ty;
        bt.anx += fabsf(tx);
        bt.any += fabsf(ty);
        bt.fp += ch.CPH[i];
        bt.afp += fabsf(ch.CPH[i]);
        bt.sym += nmx[i];
    }
    for (int q = r; q < nr; q += L) {
        const float tp = (float)ch.RPW[q], ta = (float)ch.RANG[q];
        bt.pw += tp;
        bt.ang += ta;
        bt.aang += fabsf(ta);
    }
    int kcl = 0;
    for (int ci = r; ci < c; ci += L) {
        const float4 A = ch.CLA[ci];
        for (int w = 0; w < ch.W; ++w) {
            uint64_t word = ch.NZ[ci * ch.W + w];
            while (word) {
                const int j = w * 64 + __builtin_ctzll(word);
                word &= word - 1;
                bt.cl -= overlap(A, obj_box(ch, j));
                ++kcl;
            }
        }
    }
    for (int e = r; e < c + n; e += L) {
        if ((ch.SAM[e >> 5] >> (e & 31)) & 1u) {
            const float4 v = sa_entry(ch, c, e);
            bt.sa -= (v.x + v.y) + (v.z + v.w);
        }
    }
    bt.kcl = kcl;
    bt.k = max(max((n + L - 1) / L, (nr + L - 1) / L), 4 * ((c + n + L - 1) / L));  // uniform
    ncl = group_sum<L>(kcl);
    return bt;
}

// ---- proposal (propose(), Kernel.cu:566-704) in place ---------------------------------------

__device__ __forceinline__ DBackup read_obj(const DeltaPtrs& ch, int k) {
    DBackup b;
    b.k = k;
    b.w = ch.CPH[k];
    b.x = ch.X[k];
    b.y = ch.Y[k];
    b.ry = ch.RY[k];
    return b;
}

// New pose of object k (its FocalPoint term is refreshed separately).
__device__ __forceinline__ void write_pose(const DeltaPtrs& ch, int k, double x, double y,
                                           double ry) {
    ch.X[k] = x;
    ch.Y[k] = y;
    ch.RY[k] = ry;
    float* p = &ch.P[k].xf;
    p[0] = (float)x;
    p[1] = (float)y;
    p[2] = (float)ry;
}

template <class Rng>
__device__ int2 propose(Rng& rng, const DevRoom& rm, const unsigned char* frozen,
                        const DeltaPtrs& ch, bool writer) {
    const int n = rm.n;
    const int mode = rand_int(rng, 2, 0);
    if (mode == 0) {  // translate, Kernel.cu:595-632
        const int k = pick_object(rng, n, frozen);
        float dx = rng.normal();
        dx = dx * rm.sx;
        float dy = rng.normal();
        dy = dy * rm.sy;
        const DBackup b0 = read_obj(ch, k);
        double x = b0.x, y = b0.y;
        if (x + (double)dx > rm.rmax_x) x = rm.rmax_x;
        else if (x + (double)dx < rm.rmin_x) x = rm.rmin_x;
        else x = x + (double)dx;
        if (y + (double)dy > rm.rmax_y) y = rm.rmax_y;
        else if (y + (double)dy < rm.rmin_y) y = rm.rmin_y;
        else y = y + (double)dy;
        if (writer) {
            ch.aux->b[0] = b0;
            ch.aux->nb = 1;
            ch.aux->swap_a = -1;
            write_pose(ch, k, x, y, b0.ry);
        }
        return make_int2(k, -1);
    }
    if (mode == 1) {  // rotate, Kernel.cu:634-653
        const int k = pick_object(rng, n, frozen);
        float dr = rng.normal();
        dr = (float)((double)dr * kSigmaT);
        const DBackup b0 = read_obj(ch, k);
        double ry = b0.ry + (double)dr;
        if (ry < 0) ry = ry + kTwoPI;
        else if (ry > kTwoPI) ry = ry - kTwoPI;
        if (writer) {
            ch.aux->b[0] = b0;
            ch.aux->nb = 1;
            ch.aux->swap_a = -1;
            write_pose(ch, k, b0.x, b0.y, ry);
        }
        return make_int2(k, -1);
    }
    // swap, Kernel.cu:655-703: object 1's pose travels through float temporaries.
    if (n < 2) {
        if (writer) {
            ch.aux->nb = 0;
            ch.aux->swap_a = -1;
        }
        return make_int2(-1, -1);
    }
    const int ka = pick_object(rng, n, frozen);
    const int kb = pick_object(rng, n, frozen);
    if (writer) {
        const DBackup b0 = read_obj(ch, ka);
        const DBackup b1 = read_obj(ch, kb);
        ch.aux->b[0] = b0;
        ch.aux->b[1] = b1;
        ch.aux->nb = 2;
        ch.aux->swap_a = ka;
        ch.aux->swap_b = kb;
        write_pose(ch, ka, b1.x, b1.y, b1.ry);
        write_pose(ch, kb, (double)(float)b0.x, (double)(float)b0.y, (double)(float)b0.ry);
    }
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

// ---- the ordered sums (Costs(), Kernel.cu:516-549) -----------------------------------------

// Lane k < 8 of the chain walks sum k in the reference's order from the cached terms: 0/1
// VisualBalance area*x, area*y (double terms, float accumulators, :200-201); 2 FocalPoint
// (float terms, double accumulator, :277); 3 Symmetry (float, float, :314); 4 Clearance and
// 5 SurfaceArea (float, float); 6/7 PairWise and PairWiseAngle (double, double). Each step is
// rn_d(acc + v) with v the (negated where the reference subtracts) term, rounded on to float
// for the float accumulators. Every lane reads three streams of NP entries -- multiplier m,
// double d, float f -- and adds v = m * d + f; the streams a sum does not use are ones or
// zeros, and each sequence is zero past its end, so v is the reference's term exactly.
// Sums list terms [from, to) of `fs` (the float list of lane k = 4 or 5) into the float
// accumulator a, four at a time: the reference's float accumulator with float terms, so the
// double-rounded add of the dense walk equals the plain fp32 add (53 >= 2 * 24 + 2 bits). The
// entries up to round4(to) are zero (x + 0 == x).
// The next four terms are loaded before the current four are added, so the LDS latency
// overlaps the dependent adds (these walks run ~1,000 terms at N = 256 on few waves per SIMD).
__device__ __forceinline__ float list_walk(const float* fs, int from, int to, float a) {
    if (from >= to) return a;
    float4 q = *reinterpret_cast<const float4*>(fs + from);
    for (int l = from; l < to; l += 4) {
        const float4 nq = (l + 4 < to) ? *reinterpret_cast<const float4*>(fs + l + 4) : q;
        a = a + q.x;
        a = a + q.y;
        a = a + q.z;
        a = a + q.w;
        q = nq;
    }
    return a;
}

template <int L>
__device__ void replay(const DeltaPtrs& ch, int n, const float* nmx, int cnt_cl, int cnt_sa,
                       int r, int gbase, float out[8]) {
    const DevRoom& rm = *ch.rm;
    const int k = r;
    const float* ms = ch.ONES;
    const double* ds = ch.ZERO;
    const float* fs = reinterpret_cast<const float*>(ch.ZERO);
    int lim = ch.NP;  // this lane's stream length; past it the lane reads ones / zeros
    if (k < 2) {
        ms = ch.AREA;
        ds = k == 0 ? ch.X : ch.Y;
    } else if (k == 2) {
        fs = ch.CPH;
    } else if (k == 3) {
        fs = nmx;
    } else if (k == 4) {
        fs = ch.LCL;
    } else if (k == 5) {
        fs = ch.LSA;
    } else if (k == 6) {
        ds = ch.RPW;
        lim = ch.NR;
    } else if (k == 7) {
        ds = ch.RANG;
        lim = ch.NR;
    }
    double accf = 0.0, accd = 0.0;  // float- and double-accumulated walks of the same terms
    for (int l0 = 0; l0 < ch.DL; l0 += 4) {
        const bool in = l0 < lim;
        const float* msl = in ? ms : ch.ONES;
        const double* dsl = in ? ds : ch.ZERO;
        const float* fsl = in ? fs : reinterpret_cast<const float*>(ch.ZERO);
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            v[u] = (double)msl[l0 + u] * dsl[l0 + u] + (double)fsl[l0 + u];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            accd = accd + v[u];
            accf = (double)(float)(accf + v[u]);
        }
    }
    // Clearance / SurfaceArea lists longer than NP: their tails, then (lists longer than the
    // buffer, rare) further windows rebuilt in place.
    const int cnt = k == 4 ? cnt_cl : (k == 5 ? cnt_sa : 0);
    const int cap = k == 4 ? ch.cap_cl : ch.cap_sa;
    float af = (float)accf;
    const int tail = (min(cnt, cap) + 3) & ~3;
    if (tail > ch.NP) af = list_walk(fs, ch.NP, tail, af);
    for (int lo = ch.cap_cl; lo < cnt_cl; lo += ch.cap_cl) {
        wave_sync();
        build_cl_list<L>(ch, rm.c, r, lo);
        const int m = min(ch.cap_cl, cnt_cl - lo);
        for (int l = m + r; l < ((m + 3) & ~3); l += L) ch.LCL[l] = 0.0f;
        wave_sync();
        if (k == 4) af = list_walk(ch.LCL, 0, (m + 3) & ~3, af);
    }
    for (int lo = ch.cap_sa; lo < cnt_sa; lo += ch.cap_sa) {
        wave_sync();
        build_sa_list<L>(ch, n, rm.c, r, lo);
        const int m = min(ch.cap_sa, cnt_sa - lo);
        for (int l = m + r; l < ((m + 3) & ~3); l += L) ch.LSA[l] = 0.0f;
        wave_sync();
        if (k == 5) af = list_walk(ch.LSA, 0, (m + 3) & ~3, af);
    }
    accf = (double)af;
    const bool acc_float = (k == 0 || k == 1 || k == 3 || k == 4 || k == 5);
    const double acc = acc_float ? accf : accd;
    const float nx = (float)grp_get<L>(acc, 0, gbase);
    const float ny = (float)grp_get<L>(acc, 1, gbase);
    const double fp = grp_get<L>(acc, 2, gbase);
    const float sym = (float)grp_get<L>(acc, 3, gbase);
    const float cl = (float)grp_get<L>(acc, 4, gbase);
    const float sa = (float)grp_get<L>(acc, 5, gbase);
    const double pw = grp_get<L>(acc, 6, gbase);
    const double ang = grp_get<L>(acc, 7, gbase);
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

// ---- the kernel ---------------------------------------------------------------------------

template <int L, bool XW, bool TRACK>
// Up to 8 waves per workgroup: at large N one workgroup per CU holds every resident chain, so
// the room tables staged in LDS are paid for once per CU.
__global__ void __launch_bounds__(512) mh_delta_kernel(LaunchArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int G = 64 / L;
    const DeltaLds& lay = a.dlay;
    const int n = a.rm.n, c = a.rm.c, nr = a.rm.r;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane / L;
    const int r = lane % L;
    const int gbase = g * L;
    const int waves_per_wg = blockDim.x >> 6;

    ObjConst* objc_l = reinterpret_cast<ObjConst*>(lds + lay.h_obj);
    ClrConst* clrc_l = reinterpret_cast<ClrConst*>(lds + lay.h_clr);
    RelConst* relc_l = reinterpret_cast<RelConst*>(lds + lay.h_rel);
    unsigned char* frozen = lds + lay.h_frz;
    DevRoom* rm_l = reinterpret_cast<DevRoom*>(lds + lay.h_room);
    for (int i = threadIdx.x; i < n; i += blockDim.x) objc_l[i] = a.objc[i];
    for (int i = threadIdx.x; i < c; i += blockDim.x) clrc_l[i] = a.clrc[i];
    for (int i = threadIdx.x; i < nr; i += blockDim.x) relc_l[i] = a.relc[i];
    for (int i = threadIdx.x; i <= n; i += blockDim.x) frozen[i] = (i < n) ? (a.objc[i].frozen != 0) : 1;
    if (threadIdx.x == 0) *rm_l = a.rm;
    {
        float* area = reinterpret_cast<float*>(lds + lay.h_area);
        float* ones = reinterpret_cast<float*>(lds + lay.h_ones);
        double* zero = reinterpret_cast<double*>(lds + lay.h_zero);
        for (int i = threadIdx.x; i < lay.DL; i += blockDim.x) {
            area[i] = i < n ? a.objc[i].area : 0.0f;
            ones[i] = 1.0f;
            zero[i] = 0.0;
        }
    }
    __syncthreads();

    const int64_t chain = ((int64_t)blockIdx.x * waves_per_wg + wave) * G + g;
    // Chains past the end still take part in the wave's collectives (group-local only), but
    // never load or store chain state.
    if (((int64_t)blockIdx.x * waves_per_wg + wave) * G >= a.n_chains) return;
    const bool live = chain < a.n_chains;

    // The per-chain LDS addresses are computed into VGPRs (an opaque v_mov), not kept in SGPRs:
    // this kernel is bound by LDS per chain, not registers, and the scalar file was spilling.
    int boff = lay.hdr + (wave * G + g) * lay.stride;
    asm volatile("v_mov_b32 %0, %1" : "=v"(boff) : "v"(boff));
    unsigned char* base = lds + boff;
    DeltaPtrs ch;
    ch.objc = objc_l;
    ch.clrc = clrc_l;
    ch.relc = relc_l;
    ch.rm = rm_l;
    ch.AREA = reinterpret_cast<const float*>(lds + lay.h_area);
    ch.ONES = reinterpret_cast<const float*>(lds + lay.h_ones);
    ch.ZERO = reinterpret_cast<const double*>(lds + lay.h_zero);
    ch.X = reinterpret_cast<double*>(base + lay.X);
    ch.Y = reinterpret_cast<double*>(base + lay.Y);
    ch.RY = reinterpret_cast<double*>(base + lay.RY);
    ch.P = reinterpret_cast<ObjP*>(base + lay.P);
    ch.CPH = reinterpret_cast<float*>(base + lay.CPH);
    const int np = lay.NP;
    ch.RB[0] = RowBuf{reinterpret_cast<float*>(base + lay.RMX), reinterpret_cast<int*>(base + lay.RMA)};
    ch.RB[1] = RowBuf{ch.RB[0].nmx + np, ch.RB[0].arg + np};
    ch.CLA = reinterpret_cast<float4*>(base + lay.CLA);
    ch.NZ = reinterpret_cast<uint64_t*>(base + lay.NZ);
    ch.SAM = reinterpret_cast<uint32_t*>(base + lay.SAM);
    ch.SAMB = reinterpret_cast<uint32_t*>(base + lay.SAMB);
    ch.RPW = reinterpret_cast<double*>(base + lay.RPW);
    ch.RANG = reinterpret_cast<double*>(base + lay.RANG);
    ch.LCL = reinterpret_cast<float*>(base + lay.LCL);
    ch.LSA = reinterpret_cast<float*>(base + lay.LSA);
    ch.aux = reinterpret_cast<DeltaAux*>(base + lay.AUX);
    ch.W = lay.W;
    ch.SW = lay.SW;
    ch.cap_cl = lay.cap_cl;
    ch.cap_sa = lay.cap_sa;
    ch.NP = np;
    ch.NR = lay.NR;
    ch.DL = lay.DL;
    const int64_t cidx = live ? chain : 0;
    ch.zrr = a.st + cidx * (int64_t)(F_COUNT * n) + F_Z * n;
    const int nrp = lay.NR;  // relationship stream length

    // Stage the configuration, zero the streams past their ends, build every cache.
    const double* src = a.st + cidx * (int64_t)(F_COUNT * n);
    for (int i = r; i < np; i += L) {
        double x = 0.0, y = 0.0;
        if (i < n) {
            x = src[F_X * n + i];
            y = src[F_Y * n + i];
            const double ry = src[F_RY * n + i];
            ch.RY[i] = ry;
            ObjP p;
            p.xf = (float)x;
            p.yf = (float)y;
            p.rotYf = (float)ry;
            p.pad = 0.0f;
            ch.P[i] = p;
        }
        ch.X[i] = x;
        ch.Y[i] = y;
        ch.CPH[i] = 0.0f;
        ch.RB[0].put(i, RowMax{0.0f, -1});
        ch.RB[1].put(i, RowMax{0.0f, -1});
    }
    for (int q = r; q < nrp; q += L) {
        ch.RPW[q] = 0.0;
        ch.RANG[q] = 0.0;
    }
    for (int w = r; w < ch.SW; w += L) ch.SAM[w] = 0u;
    wave_sync();
    int wild = 0;
    for (int i = r; i < n; i += L) {
        ch.CPH[i] = -focal_cos(*rm_l, ch.P[i]);
        wild += wild_pose(ch.X[i], ch.Y[i], ch.RY[i]) ? 1 : 0;
    }
    int wild_cnt = group_sum<L>(wild);
    for (int e = r; e < c + n; e += L)
        if (nonzero4(sa_entry(ch, c, e))) sam_put(ch, e, true);
    for (int ci = r; ci < c; ci += L) ch.CLA[ci] = cla_box(ch, ci);
    wave_sync();
    for (int ci = 0; ci < c; ++ci) nz_row<L>(ch, n, ci, r, gbase);
    rels_delta<L>(ch, nr, -2, -1, r);
    for (int i = 0; i < n; ++i) {
        const RowMax s = scan_row<L>(ch, n, i, wild_cnt > 0, r, gbase);
        if (r == (i % L)) ch.RB[0].put(i, s);
    }
    wave_sync();

    const ChainMeta m0 = a.meta[cidx];
    const bool writer = live && r == 0;
    float cur_total = m0.costs[0];
    if (writer)
        for (int k = 0; k < 8; ++k) ch.aux->cur[k] = m0.costs[k];
    typename RngOf<XW, L>::type rng;
    rng_load(rng, a, cidx, m0);
    uint64_t accepted = m0.accepted;
    float best_total = m0.best_total;
    double beta = kBeta;
    if constexpr (TRACK)  // (the extended variants also carry parallel tempering)
        if (a.n_temps > 1) beta = a.ladder[m0.rung];
    int rc = 0;  // which RM buffer holds the current rows
#if MH_STAMPS
    unsigned long long cyc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_last;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_last) :: "memory");
#endif

#pragma clang loop unroll(disable)
    for (int it = 0; it < a.iterations; ++it) {
        for (int w = r; w < ch.SW; w += L) ch.SAMB[w] = ch.SAM[w];
        rng_prepare(rng);
        const int2 kk = propose(rng, *rm_l, frozen, ch, writer);
        const int ka = kk.x, kb = kk.y;
        wave_sync();
        // Objects ka (lane 0) and kb (lane 1): FocalPoint term, SurfaceArea bits, wildness.
        int dwild = 0;
        if (r < 2) {
            const int k = r == 0 ? ka : kb;
            if (k >= 0) {
                const ObjP p = ch.P[k];
                ch.CPH[k] = -focal_cos(*rm_l, p);
                sam_put(ch, c + k, nonzero4(comp_overlaps(*rm_l, shape_box(ch.objc[k].off, p.xf, p.yf))));
                if (k < c)
                    sam_put(ch, k, nonzero4(comp_overlaps(*rm_l, shape_box(ch.clrc[k].shape, p.xf, p.yf))));
                const DBackup& ob = ch.aux->b[r];
                dwild = (wild_pose(ch.X[k], ch.Y[k], ch.RY[k]) ? 1 : 0) -
                        (wild_pose(ob.x, ob.y, ob.ry) ? 1 : 0);
            }
        }
        const int wild_star = wild_cnt + __shfl(dwild, gbase) + __shfl(dwild, gbase + 1);
        wave_sync();
        DSTAMP(0);
        clearance_delta<L>(ch, n, c, ka, kb, r, gbase);
        DSTAMP(1);
        rels_delta<L>(ch, nr, ka, kb, r);
        DSTAMP(2);
        const RowBuf cur = rc ? ch.RB[1] : ch.RB[0];  // (no dynamic indexing: keeps ch in VGPRs)
        const RowBuf nxt = rc ? ch.RB[0] : ch.RB[1];
        symmetry_delta<L>(ch, n, cur, nxt, ka, kb, wild_star > 0, r, gbase);
        wave_sync();
        DSTAMP(3);
        // Plain chains, one per wavefront: Accept's uniform (the next draw after the proposal's,
        // Kernel.cu:710) is drawn first, and a proposal the rejection bound already rejects
        // skips the term lists and the replay.
        constexpr bool FASTD = !TRACK && L == 64;
        bool fast_rej = false;
        float u_acc = 0.0f;
        if constexpr (FASTD) {
            u_acc = rng.uniform();
            int ncl;
            const BoundTerms bt = delta_bound_terms<L>(ch, n, c, nr, nxt.nmx, r, ncl);
            fast_rej = certain_reject(*rm_l, n, c, nr, ncl, bt, u_acc, cur_total);
        }
        float sc[8];
        if (!fast_rej) {
        const int cnt_cl = build_cl_list<L>(ch, c, r, 0);
        const int cnt_sa = build_sa_list<L>(ch, n, c, r, 0);
        // zero past each list's end: to NP for the dense walk, to round4 for the list walk
        const int zcl = max(np, (min(cnt_cl, ch.cap_cl) + 3) & ~3);
        const int zsa = max(np, (min(cnt_sa, ch.cap_sa) + 3) & ~3);
        for (int l = min(cnt_cl, ch.cap_cl) + r; l < zcl; l += L) ch.LCL[l] = 0.0f;
        for (int l = min(cnt_sa, ch.cap_sa) + r; l < zsa; l += L) ch.LSA[l] = 0.0f;
        wave_sync();
        DSTAMP(4);
#if MH_STAMPS > 1
        if (r == 0 && live) {
            atomicAdd(&g_delta_counts[0], (unsigned long long)cnt_cl);
            atomicAdd(&g_delta_counts[1], (unsigned long long)cnt_sa);
            atomicAdd(&g_delta_counts[2], (unsigned long long)(cnt_cl > ch.cap_cl));
            atomicAdd(&g_delta_counts[3], (unsigned long long)(cnt_sa > ch.cap_sa));
        }
#endif
        replay<L>(ch, n, nxt.nmx, cnt_cl, cnt_sa, r, gbase, sc);
        DSTAMP(5);
        }
        // Best-of-chain: star is judged before Accept, Kernel.cu:808-816.
        if constexpr (TRACK) {
            if (a.track != TRACK_OFF && best_improves(a.track, sc[0], best_total)) {
                best_total = sc[0];
                if (live) save_best(ch, a.best + cidx * (int64_t)(F_COUNT * n), n, r, L);
            }
        }
        bool acc;
        if constexpr (TRACK) acc = accept_at(rng, sc[0], cur_total, beta);
        else if constexpr (FASTD)
            acc = !fast_rej &&
                  u_acc < accept_threshold(kBeta * ((double)sc[0] - (double)cur_total));
        else acc = accept(rng, sc[0], cur_total);
        if (acc) {
            cur_total = sc[0];
            ++accepted;
            rc ^= 1;
            wild_cnt = wild_star;
            if (writer) {
                for (int k = 0; k < 8; ++k) ch.aux->cur[k] = sc[k];
                commit_swap_zrr(ch, n);
            }
            wave_sync();
        } else {
            if (writer) {
                const int nb = ch.aux->nb;
                for (int q = nb - 1; q >= 0; --q) {
                    const DBackup b = ch.aux->b[q];
                    write_pose(ch, b.k, b.x, b.y, b.ry);
                    ch.CPH[b.k] = b.w;
                }
            }
            for (int w = r; w < ch.SW; w += L) ch.SAM[w] = ch.SAMB[w];
            wave_sync();
            clearance_delta<L>(ch, n, c, ka, kb, r, gbase);
            rels_delta<L>(ch, nr, ka, kb, r);
            wave_sync();
        }
        DSTAMP(6);
    }
#if MH_STAMPS
    if (lane == 0)
        for (int k = 0; k < 8; ++k) atomicAdd(&g_delta_cycles[k], cyc[k]);
#endif

    if (writer) {
        ChainMeta m;
        m.draws = rng.draws;
        m.accepted = accepted;
        m.bm_has = rng.bm_has;
        m.bm_val = rng.bm_val;
        rng_save(rng, a, chain);
        for (int k = 0; k < 8; ++k) m.costs[k] = ch.aux->cur[k];
        m.best_total = best_total;
        m.rung = m0.rung;
        a.meta[chain] = m;
    }
    if (live) {
        double* dst = a.st + chain * (int64_t)(F_COUNT * n);
        for (int i = r; i < n; i += L) {
            dst[F_X * n + i] = ch.X[i];
            dst[F_Y * n + i] = ch.Y[i];
            dst[F_RY * n + i] = ch.RY[i];
        }
    }
}

template <int L>
hipError_t launch_delta_l(const LaunchArgs& a, int waves_per_wg, hipStream_t stream) {
    constexpr int G = 64 / L;
    const int64_t chains_per_wg = (int64_t)waves_per_wg * G;
    const int64_t blocks = (a.n_chains + chains_per_wg - 1) / chains_per_wg;
    const size_t lds = (size_t)a.dlay.hdr + (size_t)waves_per_wg * G * a.dlay.stride;
    const dim3 grid((unsigned)blocks), block((unsigned)(64 * waves_per_wg));
    if (a.rng == RNG_CURAND_XORWOW)  // (tracking compiled in, switched at run time)
        hipLaunchKernelGGL((mh_delta_kernel<L, true, true>), grid, block, lds, stream, a);
    else if (a.track != TRACK_OFF || a.n_temps > 1)
        hipLaunchKernelGGL((mh_delta_kernel<L, false, true>), grid, block, lds, stream, a);
    else
        hipLaunchKernelGGL((mh_delta_kernel<L, false, false>), grid, block, lds, stream, a);
    return hipGetLastError();
}

}  // namespace

#if MH_STAMPS
extern "C" __attribute__((visibility("default"))) int mh_debug_delta_cycles(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_delta_cycles), sizeof(unsigned long long) * 8) !=
        hipSuccess)
        return -1;
    return hipMemcpyFromSymbol(out + 8, HIP_SYMBOL(g_delta_counts), sizeof(unsigned long long) * 4) ==
                   hipSuccess ? 0 : -1;
}
#endif

size_t delta_lds_bytes(const DeltaLds& lay, int L, int waves_per_wg) {
    return (size_t)lay.hdr + (size_t)waves_per_wg * (64 / L) * lay.stride;
}

// Resident workgroups per CU of the plain step kernel for a shape (registers, LDS and the
// wave limit all counted by the runtime). 0 if it does not fit.
int delta_blocks_per_cu(int L, int waves_per_wg, size_t lds_bytes) {
    int blocks = 0;
    hipError_t e = hipErrorInvalidValue;
    const int threads = 64 * waves_per_wg;
    switch (L) {
        case 8: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_delta_kernel<8, false, false>, threads, lds_bytes); break;
        case 16: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_delta_kernel<16, false, false>, threads, lds_bytes); break;
        case 32: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_delta_kernel<32, false, false>, threads, lds_bytes); break;
        default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_delta_kernel<64, false, false>, threads, lds_bytes); break;
    }
    return e == hipSuccess ? blocks : 0;
}

hipError_t launch_delta(const LaunchArgs& a, int L, int waves_per_wg, hipStream_t s) {
    if (a.n_chains <= 0) return hipSuccess;
    switch (L) {
        case 8: return launch_delta_l<8>(a, waves_per_wg, s);
        case 16: return launch_delta_l<16>(a, waves_per_wg, s);
        case 32: return launch_delta_l<32>(a, waves_per_wg, s);
        default: return launch_delta_l<64>(a, waves_per_wg, s);
    }
}

}  // namespace mh
