// mh_spec.hip -- the speculative step kernel: rooms of up to 8 objects when the chains are too
// few to fill the GPU (config 2: N = 8, 1,024 chains, one wavefront per SIMD).
//
// A chain's draws do not depend on its accept decisions: the object pick redraws on the static
// frozen flags only (Kernel.cu:598-602), Box-Muller's cached second normal advances with the
// draws alone, and Accept draws its uniform on every step (:710). So the proposals of the
// next steps are known before any of them is decided. One chain owns a workgroup of two
// or four wavefronts; the 64 lanes of each are K = 8 groups of GL = 8 lanes, and each group holds
// a copy of a configuration (lane r: object r) and evaluates one node of a tree of accept /
// reject histories (below) exactly as the reference does (Costs(), Kernel.cu:516-550, every sum
// in the reference's order): a chain wavefront the exact FocalPoint and relationship terms, a
// list wavefront symmetry and the Clearance / SurfaceArea lists, each replaying its own sums.
// The realised path through the tree commits; the result is the sequential chain bit for bit
// (every decision is Accept's on exact costs). At config 2's ~41% acceptance a 16-node batch
// commits ~4.1 steps for about one step's latency.

#include <stdint.h>

#include "mh_common.h"

#ifndef MH_SPEC_DEBUG
#define MH_SPEC_DEBUG 0  // diagnostic builds record chain 0's batches (mh_debug_spec); product 0
#endif
#if MH_SPEC_DEBUG
__device__ unsigned int g_spec_dbg[1 << 16];
__device__ unsigned int g_spec_dbg_n;
#endif
#ifndef MH_STAMPS
#define MH_STAMPS 0  // diagnostic builds: cycles per phase of a batch (tools/stamps.py)
#endif
#if MH_STAMPS
// cycles of the phases of a batch (0-11), then batches and committed steps (14, 15)
__device__ unsigned long long g_spec_cycles[16];
// per chain (the first 16,384): the loop's start and end on the 100 MHz counter, and where it ran
// (HW_ID in the low word: wave, SIMD, CU, SH, SE; XCC_ID in the high word), its batches, exact
// batches and refresh batches
__device__ unsigned long long g_spec_place[6 * 16384];
__device__ unsigned int g_spec_simd[4 * 16384];  // HW_ID of each wavefront of the chain
#define SSTAMP(k) do { __builtin_amdgcn_sched_barrier(0); unsigned long long _t; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t) :: "memory"); cyc[k] += _t - t_last; t_last = _t; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define SSTAMP(k) do { } while (0)
#endif

#if MH_CHECK
static __device__ unsigned int g_spec_ck[12];  // (check builds) the first wrong certain decision's inputs
#endif
namespace mh {
namespace {

constexpr int GL = 8;          // lanes per group: the largest room this kernel serves
constexpr int K = 8;           // groups per wavefront: tree nodes one wavefront evaluates
constexpr int RMAX = 2 * GL;   // relationship slots (two per lane)
constexpr int kNone = 31;      // "no node": the batch's incoming state, or no child
// A chain owns a workgroup of 2H wavefronts in H halves. Half h evaluates nodes K*h .. K*h+7 of
// the batch's tree: its chain wavefront (2h) applies each node's history, evaluates the exact
// FocalPoint and relationship terms and replays their sums, its list wavefront (2h+1) the
// symmetry rows and the Clearance / SurfaceArea lists and theirs; one workgroup barrier hands
// the eight sums of every node over, and both chain wavefronts (which hold the chain's state
// identically) decide the same realised path. At one chain per SIMD (config 2) the step is
// latency-bound: the split halves that critical path, and H = 2 (16 nodes, launches of at most
// four chains per CU) commits more steps per batch for about the same latency as H = 1 (8 nodes,
// two wavefronts, seven chains per CU).
// Each group's ordered-sum streams (doubles, pre-signed so that every sum is acc + term). Wave 0's:
// VisualBalance area x and area y (Kernel.cu:200-201), FocalPoint -cos(phi) (:277), PairWise and
// PairWiseAngle (:222, :249-253).
enum { S_VBX = 0, S_VBY = 8, S_FP = 16, S_PW = 24, S_ANG = 24 + RMAX, S_W0 = 24 + 2 * RMAX };
// Wave 1's: Symmetry -(row max) (:314), the non-zero Clearance terms in clearance-major order
// (:429) and the non-zero SurfaceArea terms (:463-479).
enum { S_SYM = 0, S_CL = 8, S_SA = 8 + GL * GL, S_W1 = 8 + GL * GL + 8 * GL };

// One step of the chain's stream (the draws of Kernel.cu:576-704 and Accept's, :710). A chain's
// draws do not depend on its decisions, so wave 1 parses the stream into these records ahead of
// wave 0, which only reads them: a ring of kRing records, filled a window (at most kRec steps
// of a 128-word Philox window) at a time.
constexpr int kRec = 32;   // records per window
constexpr int kRing = 64;  // ring entries (two windows)
struct StepRec {  // 32 bytes (LDS per chain decides how many chains a CU holds)
    int code;      // mode | (k1 + 1) << 2 | (k2 + 1) << 6 | h << 10: the proposal (k1 = k2 = -1:
                   // a swap of a single object draws nothing) and the Box-Muller cache flag after it
    float d1, d2;  // translate: dx, dy; rotate: the angle
    float u;       // Accept's uniform
    float bv;      // the cached second normal after the step (when h)
    unsigned int next_lo, next_hi;  // stream position of the next step's first draw
    int pad;
};
__device__ __forceinline__ int rec_mode(int code) { return code & 3; }
__device__ __forceinline__ int rec_k1(int code) { return ((code >> 2) & 15) - 1; }
__device__ __forceinline__ int rec_k2(int code) { return ((code >> 6) & 15) - 1; }
__device__ __forceinline__ int rec_h(int code) { return (code >> 10) & 1; }

struct SpecW0 {  // LDS of a half's chain wavefront
    double S[K][S_W0];            // each group's streams (batches decided on the bound: the
                                  // node's FocalPoint and relationship terms, estimates or
                                  // exact, in S_FP / S_PW / S_ANG and the angle terms'
                                  // allowances in the VisualBalance slots, for its commit)
    double RY[K][GL];             // each group's double rotY of every object (Symmetry, :305)
    double XD[K][GL], YD[K][GL];  // each group's double x, y (wave 1's symmetry and boxes)
    ObjP P[K][GL];                // each group's float pose words
    float EO[K][GL];              // (bound batches) each object's FocalPoint allowance: 0 for an
                                  // exact term, kDeltaCph for an estimate
};

struct SpecW1 {  // LDS of a half's list wavefront
    double S[K][S_W1];       // each group's streams
    float4 CLB[K][GL];       // each group's clearance boxes at their sources (:414-415)
};

// A node's bound (batches decided on the bound): the eight sums of bound_parts over its chain
// wavefront's lanes, the three its list wavefront contributes (lin, elin, alin: parts 4-6), and
// the node's PairWise estimate flag (pwx, as a float).
constexpr int kBS = 12;
template <int H>
struct SpecShared {  // LDS of the chain shared by its wavefronts
    double SUM[2][K * H][8];  // each node's eight sums (double-buffered by batch parity)
    float BS[K * H][kBS];     // each node's bound sums (written before the sums barrier, read
                              // after it and before the next views barrier)
    StepRec ring[kRing];  // the step records (wave 1 writes, the chain wavefronts read)
    unsigned int wd[128];  // the 128-word window of the Philox stream being parsed (wave 1)
    unsigned int produced;  // records written so far (wave 1; read by wave 0 between the barriers)
    unsigned int consumed;  // records committed so far (wave 0; read by wave 1 between them)
    int stop;             // wave 0 to the others: the chain's steps are done
    int exact;            // wave 0 to the others: this batch evaluates every node's exact costs
};

struct SpecHdr {  // LDS of the workgroup: the room tables
    RectShape objs[GL];  // off-limits rectangles (pad: area bits)
    RectShape clrs[GL];  // clearance rectangles (pad: source object)
    RelConst rel[RMAX];
    float4 re0[RMAX], re1[RMAX];  // the relationships' fp32 estimate constants (rel_est_consts)
};

constexpr int round16s(size_t v) { return (int)((v + 15) & ~(size_t)15); }
constexpr int kSpecHdrBytes = round16s(sizeof(SpecHdr));
constexpr int kSpecW0Bytes = round16s(sizeof(SpecW0));
constexpr int kSpecW1Bytes = round16s(sizeof(SpecW1));
// LDS per chain: H = 1 23.2 KB (seven chains in a CU's 160 KB), H = 2 38.8 KB (four)
template <int H>
constexpr int spec_bytes() {
    return kSpecHdrBytes + H * (kSpecW0Bytes + kSpecW1Bytes) + round16s(sizeof(SpecShared<H>));
}
static_assert(sizeof(StepRec) == 32, "StepRec");
static_assert(spec_bytes<2>() * 4 <= 160 * 1024, "four 16-node chains per CU");
static_assert(spec_bytes<1>() * 7 <= 160 * 1024, "seven 8-node chains per CU");

// A Philox word past the LDS window (frozen-object redraws only): out of line, value-only.
__device__ __attribute__((noinline)) unsigned int philox_far(uint64_t seed, uint64_t sub,
                                                             uint64_t idx) {
    return philox_word(seed, sub, idx);
}

__device__ __forceinline__ double shfl_d(double v, int src) {
    const int a = src << 2;
    return __hiloint2double(__builtin_amdgcn_ds_bpermute(a, __double2hiint(v)),
                            __builtin_amdgcn_ds_bpermute(a, __double2loint(v)));
}
__device__ __forceinline__ float shfl_f(float v, int src) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(v)));
}
__device__ __forceinline__ float readlane_f(float v, int src) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}

// FocalPointCosts term of one object, Kernel.cu:271,277 with phi() of :185-188.
__device__ __forceinline__ float focal_cos(const DevRoom& rm, float xf, float yf, float ryf) {
    const float at = atan2_f32(rm.fyf - yf, rm.fxf - xf);
    const float b = at - ryf;
    const float ph = (float)((double)b + kHalfPI);
    return cos_f32(ph);
}

// PairWise (:210-233) and PairWiseAngle (:236-263) terms of one relationship, exactly.
__device__ __forceinline__ void rel_exact(const RelConst& rc, const ObjP* P, double& tpw,
                                          double& tang) {
    double dy, dx;
    float ti;
    tpw = rel_pair(rc, P, dy, dx, ti);
    tang = rel_angle(rc, mh_atan2(dy, dx), ti);
}

__device__ __forceinline__ bool touches(const RelConst& rc, int k1, int k2) {
    auto in = [&](int o) __attribute__((always_inline)) { return o == k1 || o == k2; };
    return k1 >= 0 && (in(rc.s) || in(rc.t) || in(rc.as) || in(rc.at));
}

// Row maximum of Symmetry (Kernel.cu:301-312, floored at 0) for the reflected pose (rx, ry, rr)
// over the n objects of a group's view, screened by the fp32 estimate (mh_common.h sym_val_fast,
// whose error sym_err bounds): the leader alone is evaluated exactly when it is clear of the
// runner-up, every candidate within the bound otherwise (max is exact, so the result is the
// reference's bit for bit).
__device__ __forceinline__ float sym_row(const ObjP* P, const double* RY, int n, float rx,
                                         float ry, float rr, bool exact_mode) {
    float m1 = -INFINITY, m2 = -INFINITY;
    int j1 = -1;
    for (int j = 0; j < n; ++j) {
        const float4 q = objp_f4(P[j]);
        const float v = sym_val_fast(q, rx, ry, rr);
        m2 = __builtin_amdgcn_fmed3f(m1, m2, v);
        const bool up = v > m1;
        m1 = up ? v : m1;
        j1 = up ? j : j1;
    }
    const bool clear = j1 >= 0 && (m2 == -INFINITY || m1 - m2 > sym_err(m1, rr) + sym_err(m2, rr));
    float best = 0.0f;
    if (clear && !exact_mode) {
        const ObjP q = P[j1];
        best = fmaxf(0.0f, sym_val_exact(q.xf, q.yf, RY[j1], rx, ry, (double)rr));
    } else {
        const float thr = (exact_mode || j1 < 0) ? INFINITY : 2.0f * sym_err(fabsf(m1) + 1.0f, rr);
        for (int j = 0; j < n; ++j) {
            const ObjP q = P[j];
            const float v = sym_val_fast(objp_f4(q), rx, ry, rr);
            if (!(v < m1 - thr)) best = fmaxf(best, sym_val_exact(q.xf, q.yf, RY[j], rx, ry, (double)rr));
        }
    }
    return best;
}

// Sum of v over this lane's group of 8 (every lane of the group gets it): three DPP levels.
__device__ __forceinline__ float grp8_fsum(float v) {
    v += bfly<1>(v);
    v += bfly<2>(v);
    v += bfly<4>(v);
    return v;
}

// Appends the non-zero components of t (when `on`), in lane order within each group, to the
// group's stream at `pos` (pre-negated: the reference subtracts them); advances pos by the
// group's count.
__device__ __forceinline__ void append4(const Staged<double>& S, int& pos, float4 t, bool on,
                                        int r) {
    const int cnt = on ? (int)(t.x != 0.0f) + (int)(t.y != 0.0f) + (int)(t.z != 0.0f) +
                             (int)(t.w != 0.0f)
                       : 0;
    int tot;
    int q = pos + group_excl_scan<GL>(cnt, r, tot);
    if (on) {
        if (t.x != 0.0f) S.put(q++, -(double)t.x);
        if (t.y != 0.0f) S.put(q++, -(double)t.y);
        if (t.z != 0.0f) S.put(q++, -(double)t.z);
        if (t.w != 0.0f) S.put(q++, -(double)t.w);
    }
    pos += tot;
}

// ---- speculation trees ----------------------------------------------------------------------
// A batch evaluates the NN nodes of a prefix-closed tree of accept / reject histories. Node k
// evaluates the proposal of step t + dep(k) against the configuration its history leaves -- the
// batch's incoming state with the proposals of the steps it accepted applied in order -- and its
// Accept compares with the total of the node whose proposal that configuration is (cpar), or the
// incoming total. The realised path walks from the root by Accept's decisions until it leaves the
// tree; its steps commit. Every decision on the path is Accept's on exact costs of the
// configuration the sequential chain holds there, so any prefix-closed tree gives the sequential
// chain bit for bit; the shape only sets how many steps a batch commits: with acceptance rate p,
// the sum of its nodes' path probabilities, largest for the NN most probable histories. (Round
// 4's linear speculation is the all-reject path; at config 2's p = 0.41 it commits 2.46 steps per
// batch, the 8-node tree {root, R, A, RR, RA, AR, RRR, AA} 3.22, the 16-node tree 4.14.)
struct SpecTree {  // lane k < NN: node k; other lanes: unused
    int dep;     // its step's offset in the batch
    int hist;    // bit i set: step t + i accepted on its history (i < dep)
    int cpar;    // the node whose configuration is its current one (kNone: the incoming state)
    int cha, chr;  // the next node on an accept / a reject (kNone: none)
    int maxdep;  // (wave-uniform) the deepest node's dep
};

// The NN most probable histories for acceptance rate p, grown best-first from the root (a child
// is less probable than its parent, so the set is prefix-closed), lane k building node k: each
// round the open child of largest probability, the lowest node and its reject child first on
// ties.
template <int NN>
__device__ __forceinline__ SpecTree spec_tree(float p) {
    static_assert(NN <= 32, "nodes");
    p = fminf(fmaxf(p, 0.02f), 0.98f);
    const int lane = __lane_id();
    SpecTree t;
    float pr = lane == 0 ? 1.0f : -1.0f;
    t.dep = t.hist = 0;
    t.cpar = t.cha = t.chr = kNone;
#pragma unroll 1
    for (int k = 1; k < NN; ++k) {
        const float q0 = (lane < k && t.chr == kNone) ? pr * (1.0f - p) : -1.0f;
        const float q1 = (lane < k && t.cha == kNone) ? pr * p : -1.0f;
        const int b = q1 > q0 ? 1 : 0;
        const float q = b ? q1 : q0;
        float m = q;
#pragma unroll
        for (int off = 1; off < 32; off <<= 1) m = fmaxf(m, __shfl_xor(m, off, 32));
        const float mu = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(m)));
        const uint64_t hit = __ballot(lane < k && q == mu);
        const int bi = (int)__builtin_ctzll(hit);
        const int bb = __builtin_amdgcn_readlane(b, bi);
        const int pdp = __builtin_amdgcn_readlane(t.dep, bi);
        const int phs = __builtin_amdgcn_readlane(t.hist, bi);
        const int pcp = __builtin_amdgcn_readlane(t.cpar, bi);
        if (lane == bi) {
            if (bb) t.cha = k;
            else t.chr = k;
        }
        if (lane == k) {
            pr = mu;
            t.dep = pdp + 1;
            t.hist = phs | (bb << pdp);
            t.cpar = bb ? bi : pcp;
        }
    }
    int md = lane < NN ? t.dep : 0;
#pragma unroll
    for (int off = 1; off < 32; off <<= 1) md = max(md, __shfl_xor(md, off, 32));
    t.maxdep = __builtin_amdgcn_readfirstlane(md);
    return t;
}

// Position of the q-th set bit (q from 0) of a 16-bit mask: a branch-free binary search.
__device__ __forceinline__ int nth_bit(uint32_t m, int q) {
    int pos = 0;
    int c = __builtin_popcount(m & 0xffu);
    if (q >= c) { q -= c; m >>= 8; pos += 8; }
    c = __builtin_popcount(m & 0xfu);
    if (q >= c) { q -= c; m >>= 4; pos += 4; }
    c = __builtin_popcount(m & 0x3u);
    if (q >= c) { q -= c; m >>= 2; pos += 2; }
    if (q >= (int)(m & 1u)) pos += 1;
    return pos;
}

template <int H, bool BOUND>
__global__ void __launch_bounds__(128 * H) mh_spec_kernel(LaunchArgs a) {
    constexpr int NN = K * H;  // tree nodes per batch
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int lane = __lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int hf = wave >> 1;            // (wave-uniform) the half: nodes K*hf .. K*hf + 7
    const bool chain_wave = (wave & 1) == 0;
    const int g = lane >> 3, r = lane & 7, gbase = lane & ~7;
    const DevRoom& rm = a.rm;
    const int n = rm.n, c = rm.c, nr = rm.r;

    SpecHdr* Hd = reinterpret_cast<SpecHdr*>(lds);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        RectShape s = a.objc[i].off;
        s.pad = __float_as_int(a.objc[i].area);
        Hd->objs[i] = s;
    }
    for (int i = threadIdx.x; i < c; i += blockDim.x) {
        RectShape s = a.clrc[i].shape;
        s.pad = a.clrc[i].src;
        Hd->clrs[i] = s;
    }
    for (int i = threadIdx.x; i < nr; i += blockDim.x) {
        Hd->rel[i] = a.relc[i];
        Hd->re0[i] = a.rele[i];
        Hd->re1[i] = a.rele[nr + i];
    }
    __syncthreads();

    const int64_t chain = (int64_t)blockIdx.x;  // (the whole workgroup: one chain)
    if (chain >= a.n_chains) return;
#if MH_STAMPS
    if ((threadIdx.x & 63) == 0 && chain < 16384)  // where each of the chain's wavefronts runs
        g_spec_simd[4 * chain + (threadIdx.x >> 6)] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
#endif
    // per half: the chain wavefront's LDS, then the list wavefront's; then the shared part
    auto X0of = [&](int h) __attribute__((always_inline)) {
        return reinterpret_cast<SpecW0*>(lds + kSpecHdrBytes + h * kSpecW0Bytes);
    };
    SpecW0* X0 = X0of(hf);
    SpecW1* X1 = reinterpret_cast<SpecW1*>(lds + kSpecHdrBytes + H * kSpecW0Bytes + hf * kSpecW1Bytes);
    SpecShared<H>* SH = reinterpret_cast<SpecShared<H>*>(
        lds + kSpecHdrBytes + H * (kSpecW0Bytes + kSpecW1Bytes));
    int par = 0;                 // the batch's SUM buffer
    const ChainMeta m0 = a.meta[chain];

    if (!chain_wave) {
        // ---- The list wavefronts: per batch the symmetry rows and the Clearance / SurfaceArea
        // lists of their half's nodes. Wave 1 also writes the stream's step records ahead of the
        // chain wavefronts. They keep no chain state.
        //
        // The Philox stream (key = seed, subsequence = global id), 128 words at a time: lane i
        // holds words start + i and start + 64 + i; LDS the words and the Box-Muller pairs of
        // both. A step's draws (Kernel.cu:576-710): the mode, the picks (with frozen redraws),
        // the normals, Accept's uniform. Only the normals depend on the state before the step
        // (the cached second normal h): translate takes one pair either way (h unchanged, the
        // pair's second normal cached when h = 1), rotate one pair when h = 0 (then cached) and
        // none when h = 1, swap none. So every lane parses the steps that would start at its two
        // offsets of the window, a wave-uniform walk chains the window's steps (none of it
        // depends on a decision), and lane s writes step s's record into the ring.
        const bool producer = hf == 0;
        unsigned int fz = 1u << n;  // frozen flags, index n frozen (a pick of n is redrawn)
        for (int i = 0; i < n; ++i) fz |= (a.objc[i].frozen != 0 ? 1u : 0u) << i;
        const uint64_t seed = a.seed, sub = (uint64_t)(a.chain_offset + chain);
        uint64_t wbase = 0;
        Published<unsigned int> win{SH->wd};
        Published<StepRec> ringv{SH->ring};
        // Draws at a lane's own offset (every lane may read a different one).
        auto word_v = [&](unsigned int o) __attribute__((always_inline)) -> unsigned int {
            return o < 128 ? win[o] : philox_far(seed, sub, wbase + o);
        };
        auto rand_v = [&](unsigned int& o, int mx) __attribute__((always_inline)) {  // generateRandomIntInRange, Kernel.cu:566-574
            float u = rocrand_device::detail::uniform_distribution(word_v(o++));
            u = (float)((double)u * ((double)mx + 0.999999));
            u = u + 0.0f;
            return (int)truncf(u);
        };
        auto rand_w = [&](unsigned int w, int mx) __attribute__((always_inline)) {  // the same, of a word already read
            float u = rocrand_device::detail::uniform_distribution(w);
            u = (float)((double)u * ((double)mx + 0.999999));
            u = u + 0.0f;
            return (int)truncf(u);
        };
        // The mode and picks of a step starting at window offset o0 (< 124), packed with the
        // offset after them (Kernel.cu:582, 598-602, 657-671; index n counts as frozen).
        auto parse = [&](unsigned int o0, int& k1, int& k2) __attribute__((always_inline)) -> int {
            const unsigned int wa = win[o0], wb = win[o0 + 1], wc = win[o0 + 2];
            unsigned int o = o0 + 1;
            const int md = rand_w(wa, 2);
            k1 = -1;
            k2 = -1;
            if (md != 2 || n >= 2) {
                k1 = rand_w(wb, n - 1);
                o = o0 + 2;
                while ((fz >> k1) & 1u) k1 = rand_v(o, n - 1);
                if (md == 2) {
                    k2 = rand_w(o == o0 + 2 ? wc : word_v(o), n - 1);
                    ++o;
                    while ((fz >> k2) & 1u) k2 = rand_v(o, n - 1);
                }
            }
            return md | (int)(o << 2);
        };
        // The producer's position: where the next unparsed step starts, the cache before it.
        uint64_t ppos = m0.draws;
        int ph = m0.bm_has;
        float pbv = m0.bm_val;
        unsigned int prod = 0;  // records written
        // One window at ppos: its words and Box-Muller pairs, its steps' records into the ring
        // at prod, prod + 1, ...
        auto produce = [&]() __attribute__((always_inline)) {
            wbase = ppos;
            const unsigned int w0 = philox_word(seed, sub, wbase + (uint64_t)lane);
            const unsigned int w1 = philox_word(seed, sub, wbase + 64 + (uint64_t)lane);
            const Staged<unsigned int> w = restage(win);  // (every lane's reads are done)
            w.put(lane, w0);
            w.put(64 + lane, w1);
            win = publish(w);
            // the steps that would start at offsets lane and 64 + lane (past 123: not parsed)
            int ka_lo, kb_lo, ka_hi = -1, kb_hi = -1;
            const int pk_lo = parse((unsigned int)lane, ka_lo, kb_lo);
            int pk_hi = 3;
            if (lane < 60) pk_hi = parse(64u + (unsigned int)lane, ka_hi, kb_hi);
            // the walk: (offset, h, the step whose pair's second normal is cached: -1 = pbv),
            // wave-uniform; lane s keeps step s's start, h, cache and next start
            unsigned int wo = 0u, s_go = 0u, s_next = 1u;
            int wh = __builtin_amdgcn_readfirstlane(ph), wcs = -1, s_h = 0, s_cs = -1;
            int s = 0;
#pragma clang loop unroll(disable)
            for (; s < kRec && wo < 124u; ++s) {
                const int i = __builtin_amdgcn_readfirstlane((int)wo);
                const int vl = __builtin_amdgcn_readlane(pk_lo, i & 63);
                const int vh = __builtin_amdgcn_readlane(pk_hi, i & 63);
                const int v = i < 64 ? vl : vh;
                const int md = v & 3;
                const unsigned int pa = (unsigned int)v >> 2;
                s_go = lane == s ? wo : s_go;
                s_h = lane == s ? wh : s_h;
                s_cs = lane == s ? wcs : s_cs;
                const bool tr_ = md == 0, ro = md == 1;  // translate, rotate (swap: 2)
                const bool pair = tr_ || (ro && !wh);    // the step takes a Box-Muller pair
                wcs = (tr_ && wh) || (ro && !wh) ? s : wcs;  // ... and caches its second
                wo = pa + (pair ? 3u : 1u);
                wh = ro ? !wh : wh;
                s_next = lane == s ? wo : s_next;
            }
            const int nrec = s;
            // lane s: step s's record from the parsing lane, its Box-Muller pair (only the steps
            // that take one: at most one per lane), the cached normal from the step that cached
            // it, and Accept's uniform
            StepRec R;
            {
                const int src = (int)(s_go & 63u) << 2;
                const bool hi = s_go >= 64u;
                const int md_lo = __builtin_amdgcn_ds_bpermute(src, pk_lo);
                const int md_hi = __builtin_amdgcn_ds_bpermute(src, pk_hi);
                const int a_lo = __builtin_amdgcn_ds_bpermute(src, ka_lo);
                const int a_hi = __builtin_amdgcn_ds_bpermute(src, ka_hi);
                const int b_lo = __builtin_amdgcn_ds_bpermute(src, kb_lo);
                const int b_hi = __builtin_amdgcn_ds_bpermute(src, kb_hi);
                const int v = hi ? md_hi : md_lo;
                const int mode = v & 3, k1 = hi ? a_hi : a_lo, k2 = hi ? b_hi : b_lo;
                const unsigned int pa = (unsigned int)v >> 2;
                const bool pair = lane < nrec && (mode == 0 || (mode == 1 && !s_h));
                float2 z = make_float2(0.0f, 0.0f);
                if (pair) z = box_muller_inl(word_v(pa), word_v(pa + 1));
                const float zc_c = shfl_f(z.y, s_cs < 0 ? 0 : s_cs);  // (every lane active)
                const float bvi = s_cs < 0 ? pbv : zc_c;
                const unsigned int wu = word_v(s_next - 1);
                const float zs = z.x, zc = z.y;
                R.d1 = 0.0f;
                R.d2 = 0.0f;
                int h = s_h;
                R.bv = bvi;
                if (mode == 0) {  // translate, Kernel.cu:595-632
                    R.d1 = (s_h ? bvi : zs) * rm.sx;
                    R.d2 = (s_h ? zs : zc) * rm.sy;
                    R.bv = zc;
                } else if (mode == 1) {  // rotate, :634-653
                    const float dr = s_h ? bvi : zs;
                    R.d1 = (float)((double)dr * kSigmaT);
                    h = !s_h;
                    R.bv = s_h ? bvi : zc;
                }
                R.code = mode | ((k1 + 1) << 2) | ((k2 + 1) << 6) | (h << 10);
                R.u = rocrand_device::detail::uniform_distribution(wu);  // Accept, :710
                const uint64_t nx = wbase + s_next;
                R.next_lo = (unsigned int)nx;
                R.next_hi = (unsigned int)(nx >> 32);
                R.pad = 0;
            }
            const Staged<StepRec> rs = restage(ringv);
            if (lane < nrec) rs.put((int)((prod + (unsigned int)lane) % (unsigned int)kRing), R);
            ringv = publish(rs);
            // the stream after the window's last step
            const int lastl = nrec - 1;
            ppos = ((uint64_t)(unsigned int)__builtin_amdgcn_readlane((int)R.next_hi, lastl) << 32) |
                   (unsigned int)__builtin_amdgcn_readlane((int)R.next_lo, lastl);
            ph = rec_h(__builtin_amdgcn_readlane(R.code, lastl));
            pbv = readlane_f(R.bv, lastl);
            prod += (unsigned int)nrec;
        };
        const Staged<unsigned int> PROD{&SH->produced};
        if (producer) {
            produce();
            produce();
            if (lane == 0) PROD.put(0, prod);
        }
        __syncthreads();  // (the chain wavefronts start with these records)
        unsigned int cons_seen = 0;  // records wave 0 had committed, as read between the barriers
        const Staged<double> Sst{X1->S[g]};
        const Staged<float4> CLBst{X1->CLB[g]};
#pragma clang loop unroll(disable)
        for (;;) {
            // the ring has room for a window (the chain wavefronts read records below cons_seen
            // no more)
            if (producer && prod + (unsigned int)kRec <= cons_seen + (unsigned int)kRing) {
                produce();
                if (lane == 0) PROD.put(0, prod);
            }
            const auto pv = receive_workgroup(X0->P[g], X0->RY[g], X0->XD[g], X0->YD[g]);
            if (SH->stop) break;
            cons_seen = SH->consumed;
            // (check builds evaluate the exact costs and the bound of every batch)
            const bool exact_b = !BOUND || SH->exact != 0 || MH_CHECK;
            const bool bound_b = BOUND && (SH->exact == 0 || MH_CHECK);
            const ObjP* Pg = pv.a.ptr();
            const int ro = r < n ? r : 0;
            const double sx = pv.c[ro], sy = pv.d[ro], sry = pv.b[ro];
            const float xf = Pg[ro].xf, yf = Pg[ro].yf;
            float4 box = make_float4(0.f, 0.f, 0.f, 0.f), sao = box, sac = box;
            bool wild = false;
            if (r < n) {
                box = shape_box(Hd->objs[r], xf, yf);
                sao = comp_overlaps(rm, box);  // SurfaceArea, object r (:469-480)
                wild = !(fabs(sx) < 1e15 && fabs(sy) < 1e15 && fabs(sry) < 1e15);
            }
            if (r < c) {
                const RectShape cs = Hd->clrs[r];
                const ObjP ps = Pg[cs.pad];
                CLBst.put(r, shape_box(cs, ps.xf, ps.yf));      // Clearance, :414-415
                sac = comp_overlaps(rm, shape_box(cs, xf, yf));  // SurfaceArea quirk: cfg[i], :456
            }
            // Symmetry row r, Kernel.cu:292-312.
            const bool exact_mode = group_ballot<GL>(wild, gbase) != 0;
            float rxr = 0.0f, ryr = 0.0f, rr = 0.0f;
            if (r < n) {
                double al = sx * (double)rm.ux;
                al = al + sy * (double)rm.uy;
                const float sd = (float)(2.0 * (rm.along_f - al));
                rxr = (float)(sx + (double)(sd * rm.ux));
                ryr = (float)(sy + (double)(sd * rm.uy));
                rr = (float)(rm.two_focal_rot - sry);
                if ((double)rr < -kPI) rr = (float)((double)rr + kTwoPI);
                if (exact_b)
                    Sst.put(S_SYM + r, -(double)sym_row(Pg, pv.b.ptr(), n, rxr, ryr, rr, exact_mode));
            }
            const auto sv = publish(Sst, CLBst);
            if constexpr (BOUND || MH_CHECK) {  // (the exact instance compiles none of it)
                if (bound_b) {
                    // The node's bound, this wavefront's share (bound_parts): the row maximum's fp32
                    // estimate with sym_err's allowance (max(0, .) is 1-Lipschitz, and the exact row
                    // maximum lies within the estimate's allowance of the largest estimate), the
                    // lane's column of Clearance terms in clearance order, its SurfaceArea terms.
                    BoundTerms bt{};
                    bt.k = 8;
                    if (r < n) {
                        float m1 = -INFINITY;
                        for (int j = 0; j < n; ++j)
                            m1 = fmaxf(m1, sym_val_fast(objp_f4(Pg[j]), rxr, ryr, rr));
                        const float mx = fmaxf(0.0f, m1);
                        bt.esym = sym_err(m1, rr);
                        bt.sym = -mx;
                        bt.symw = (float)(n - r) * (mx + bt.esym);  // (row r: position r)
                        float cls = 0.0f;
                        for (int i = 0; i < c; ++i) {
                            const float ov = overlap(sv.b[i], box);
                            cls += ov;
                            bt.kcl += ov != 0.0f ? 1 : 0;
                        }
                        bt.cl = -cls;
                    }
                    bt.sa = -((sac.x + sac.y + sac.z + sac.w) + (sao.x + sao.y + sao.z + sao.w));
                    int ncl = bt.kcl;  // (the node's non-zero Clearance terms)
                    ncl += __builtin_amdgcn_update_dpp(0, ncl, 0xB1, 0xF, 0xF, false);
                    ncl += __builtin_amdgcn_update_dpp(0, ncl, 0x4E, 0xF, 0xF, false);
                    ncl += __builtin_amdgcn_update_dpp(0, ncl, 0x141, 0xF, 0xF, false);
                    float part[8];
                    bound_parts(rm, n, c, nr, ncl, bt, part);
                    // a pose outside the range the symmetry estimate is proven for: no bound (NaN)
                    const float lin = exact_mode ? __builtin_nanf("") : part[4];
                    const float s4 = grp8_fsum(lin), s5 = grp8_fsum(part[5]), s6 = grp8_fsum(part[6]);
                    const Staged<float> B{SH->BS[K * hf + g]};
                    if (r == 0) {
                        B.put(8, s4);
                        B.put(9, s5);
                        B.put(10, s6);
                    }
                }
                if (!exact_b) {  // (the barrier below publishes the bound's sums)
                    publish_workgroup(Staged<double>{SH->SUM[par][K * hf + g]});
                    par ^= 1;
                    continue;
                }
            }
            // The non-zero Clearance terms, clearance-major (:408-431), and SurfaceArea terms
            // (clearances, then objects, :445-480), compacted in the reference's order.
            int ncl = 0, nsa = 0;
            for (int i = 0; i < c; ++i) {
                float4 t4 = make_float4(0.f, 0.f, 0.f, 0.f);
                if (r < n) t4.x = overlap(sv.b[i], box);
                append4(Sst.at(S_CL), ncl, t4, r < n, r);
            }
            append4(Sst.at(S_SA), nsa, sac, r < c, r);
            append4(Sst.at(S_SA), nsa, sao, r < n, r);
            const Published<double> Sv = publish(Sst);
            // Sums 3 (Symmetry), 4 (Clearance), 5 (SurfaceArea), as in the chain wavefronts'
            // replay below.
            const Staged<double> SUMst{SH->SUM[par][K * hf + g]};
            if (r >= 3 && r <= 5) {
                const int base = r == 3 ? S_SYM : r == 4 ? S_CL : S_SA;
                const int len = r == 3 ? n : r == 4 ? ncl : nsa;
                const double* src = Sv.ptr() + base;
                double acc = 0.0;
                for (int l = 0; l < len; ++l) acc = (double)(float)(acc + src[l]);
                SUMst.put(r, acc);
            }
            publish_workgroup(SUMst);
            par ^= 1;
        }
        return;
    }

    // ---- The chain wavefronts (wave 0, and wave 2 when H = 2): the same chain state in both.
    // The current configuration, in every group: lane r holds object r (z, rotX and rotZ too:
    // no cost reads them, an accepted swap exchanges them, Kernel.cu:675-700). Wave 0 alone writes
    // the shared flags and the chain's results.
    const bool lead = hf == 0;
    double* st = a.st + chain * (int64_t)(F_COUNT * n);
    double cx = 0.0, cy = 0.0, cry = 0.0, cz = 0.0, crx = 0.0, crz = 0.0;
    if (r < n) {
        cx = st[F_X * n + r];
        cy = st[F_Y * n + r];
        cry = st[F_RY * n + r];
        cz = st[F_Z * n + r];
        crx = st[F_RX * n + r];
        crz = st[F_RZ * n + r];
    }
    float cur[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) cur[k] = m0.costs[k];

    // The current configuration's per-object and per-relationship terms (carried across
    // steps; a proposal recomputes the ones it changes).
    // (LDS shared between lanes moves through Staged / Published views, mh_common.h)
    const Staged<ObjP> Pst{X0->P[g]};
    const Staged<double> RYst{X0->RY[g]};
    const Staged<double> Sall{&X0->S[0][0]};  // every group's streams (group g at g * S_W0)
    const Staged<double> XDst{X0->XD[g]}, YDst{X0->YD[g]};
    const Staged<int> STOP{&SH->stop};
    const Staged<unsigned int> CONS{&SH->consumed};
    const Staged<int> EXACT{&SH->exact};
    if (r < n) {
        ObjP p;
        p.xf = (float)cx;
        p.yf = (float)cy;
        p.rotYf = (float)cry;
        p.pad = 0.0f;
        Pst.put(r, p);
        RYst.put(r, cry);
    }
    if (lead && lane == 0) CONS.put(0, 0u);
    const Published<ObjP> P0 = publish(Pst);
    float cph = 0.0f;
    double rpw0 = 0.0, rang0 = 0.0, rpw1 = 0.0, rang1 = 0.0;
    if (r < n) cph = focal_cos(rm, (float)cx, (float)cy, (float)cry);
    if (r < nr) rel_exact(Hd->rel[r], P0.ptr(), rpw0, rang0);
    if (r + GL < nr) rel_exact(Hd->rel[r + GL], P0.ptr(), rpw1, rang1);

    __syncthreads();  // (wave 1's first records)
    const Published<StepRec> ring{SH->ring};
    unsigned int prod_seen = SH->produced;  // records wave 1 had written, read between barriers
    unsigned int cons = 0;                  // records committed
    // the stream after the last committed step (the launch's end state)
    uint64_t end_pos = m0.draws;
    int end_h = m0.bm_has;
    float end_bv = m0.bm_val;
    auto rec = [&](unsigned int i) __attribute__((always_inline)) -> const StepRec& {
        return ring[(int)(i % (unsigned int)kRing)];
    };
    // Applies to (x, y, ry), lane r's object, the proposals of the steps i < cnt for which
    // take(i) holds, in step order (Kernel.cu:576-704; each is the reference's edit of cfgStar,
    // made on the configuration it would see). Every lane must be active (the swap's shuffles).
    // The batch's records ride in registers: lane i holds record cons + i (one pair of
    // ds_read_b128 per batch), and a step's fields are lane reads, not LDS round trips on the
    // chain's critical path (config 2: ~750 cycles per applied step before).
    int r_code = 0;
    float r_d1 = 0.0f, r_d2 = 0.0f, r_u = 1.0f;
    auto apply = [&](double& x, double& y, double& ry, bool& mv, int cnt, auto take)
        __attribute__((always_inline)) {
        for (int i = 0; i < cnt; ++i) {  // (wave-uniform: the step's record)
            const bool app = take(i);
            const int qc = __builtin_amdgcn_readlane(r_code, i);
            const int qm = rec_mode(qc), q1 = rec_k1(qc), q2 = rec_k2(qc);
            const float qd1 = readlane_f(r_d1, i), qd2 = readlane_f(r_d2, i);
            if (qm == 0) {  // translate
                if (app && r == q1) {
                    mv = true;
                    if (x + (double)qd1 > rm.rmax_x) x = rm.rmax_x;
                    else if (x + (double)qd1 < rm.rmin_x) x = rm.rmin_x;
                    else x = x + (double)qd1;
                    if (y + (double)qd2 > rm.rmax_y) y = rm.rmax_y;
                    else if (y + (double)qd2 < rm.rmin_y) y = rm.rmin_y;
                    else y = y + (double)qd2;
                }
            } else if (qm == 1) {  // rotate
                if (app && r == q1) {
                    mv = true;
                    ry = ry + (double)qd1;
                    if (ry < 0) ry = ry + kTwoPI;
                    else if (ry > kTwoPI) ry = ry - kTwoPI;
                }
            } else if (q1 >= 0) {  // swap (every lane active for the shuffles)
                const int ia = gbase + q1, ib = gbase + q2;
                const double ax = shfl_d(x, ia), ay = shfl_d(y, ia), ary = shfl_d(ry, ia);
                const double bx = shfl_d(x, ib), by = shfl_d(y, ib), bry = shfl_d(ry, ib);
                // object 1 takes object 2's pose, object 2 object 1's through float temporaries
                if (app && r == q2) {
                    x = (double)(float)ax;
                    y = (double)(float)ay;
                    ry = (double)(float)ary;
                    mv = true;
                } else if (app && r == q1) {
                    x = bx;
                    y = by;
                    ry = bry;
                    mv = true;
                }
            }
        }
    };

    unsigned int accepted = 0;
    // The batch's tree (spec_tree), rebuilt every 32 batches from this launch's acceptance rate
    // (a prior of 2 accepts in 5 steps to start): lane k < NN holds node k; each group's own
    // node is K * hf + g.
    SpecTree tr;
    int my_dep = 0, my_hist = 0;
    auto set_tree = [&](float p) __attribute__((always_inline)) {
        tr = spec_tree<NN>(p);
        const int src = (K * hf + g) << 2;
        my_dep = __builtin_amdgcn_ds_bpermute(src, tr.dep);
        my_hist = __builtin_amdgcn_ds_bpermute(src, tr.hist);
    };
    set_tree(0.4f);
    unsigned int batches = 0;
    // Decisions on the bound (BOUND; mh_common.h bound_parts / bound_te): a batch first
    // bounds every node's total from fp32 estimates -- the moved objects' FocalPoint terms and the
    // touched relationships' terms as the full-evaluation kernel estimates them, the symmetry row
    // maxima as their screening estimates, the other terms exact -- and decides Accept where the
    // bound makes it certain. The realised path commits while its decisions are certain; at the
    // first open one it stops, and the next batch evaluates every node's exact costs (as every
    // batch does without the bound); when a certain acceptance left the current costs an interval,
    // that batch's last node evaluates the incoming configuration instead (a refresh), and the
    // root's decisions compare with its exact total. The carried terms may be estimates
    // (allowances efp_c, ea0_c, ea1_c: 0 when exact); an exact batch evaluates them exactly.
    float efp_c = 0.0f, ea0_c = 0.0f, ea1_c = 0.0f;
    CostIv cur_iv{cur[0], cur[0]};
    bool cur_exact = true;
    bool exact_next = !BOUND;
    // Where the bound keeps leaving nodes open -- a chain whose configuration sits near a branch of
    // an estimate, say -- its stops cost more than the bound saves, and the launch waits for that
    // chain. An open stop within 4 bound batches of the previous one doubles a run of exact
    // batches that follows it (up to 64); a later one resets it (exact_run: exact batches still to
    // run after the one the stop asks for; since_open: bound batches since the last stop).
    int exact_run = 0, backoff = 1, since_open = 0;
#if MH_STAMPS
    unsigned long long cyc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, t_last, rt0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_last) :: "memory");
    // the constant 100 MHz counter beside it: shader cycles / real time = the clock the chain ran at
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rt0) :: "memory");
    const unsigned long long t_first = t_last;
#endif
#pragma clang loop unroll(disable)
    for (int done = 0;;) {
        const bool finish = done >= a.iterations;
        if (finish && cur_exact) {  // (the list wavefronts leave their loop at this barrier)
            if (lead && lane == 0) STOP.put(0, 1);
            publish_workgroup(STOP);
            break;
        }
        // (check builds: exact costs and the bound in every batch, decisions on the exact costs)
        const bool exact_b = exact_next || exact_run > 0 || finish || !BOUND || MH_CHECK;
        const bool bound_b = !exact_b || MH_CHECK;
        // a launch ends, and an exact batch decides, with the current configuration's exact
        // costs: when a certain acceptance left them an interval, node NN - 1 evaluates the
        // incoming configuration (the tree without that node this batch)
        const bool refresh = exact_b && !cur_exact;
        if ((++batches & 31u) == 0u)
            set_tree((float)(accepted + 2u) / (float)(done + 5));
        const int dep_g = refresh && K * hf + g == NN - 1 ? -1 : my_dep;  // (-1: nothing applied)
        // steps this batch can reach: the tree's depth, the launch's remaining steps, the
        // records wave 1 has written (0: a round that only waits for it)
        const int kb = min(min(tr.maxdep + 1, a.iterations - done), (int)(prod_seen - cons));
        if (lane < kb) {
            const StepRec& q = rec(cons + (unsigned int)lane);
            r_code = q.code;
            r_d1 = q.d1;
            r_d2 = q.d2;
            r_u = q.u;
        }
        SSTAMP(0);
        // Group g's configuration: the incoming state with the proposals of the steps its
        // node's history accepted and then its own step's applied in step order.
        double sx = cx, sy = cy, sry = cry;
        bool moved = false;  // this lane's object differs from the incoming state
        apply(sx, sy, sry, moved, kb, [&](int i) __attribute__((always_inline)) {
            return i == dep_g || (i < dep_g && ((my_hist >> i) & 1));
        });
        const float xf = (float)sx, yf = (float)sy, ryf = (float)sry;
        if (r < n) {
            ObjP p;
            p.xf = xf;
            p.yf = yf;
            p.rotYf = ryf;
            p.pad = 0.0f;
            Pst.put(r, p);
            RYst.put(r, sry);
            XDst.put(r, sx);
            YDst.put(r, sy);
        }
        if (lead && lane == 0) {
            STOP.put(0, 0);
            EXACT.put(0, exact_b ? 1 : 0);
        }
        SSTAMP(1);
        const auto pv = publish_workgroup(Pst, RYst, XDst, YDst);  // (to the list wavefront too)
        SSTAMP(2);
        prod_seen = SH->produced;  // (wave 1 writes it before this barrier, never between)
        (void)pv;  // (the views are read below through Pall: every group's)
        const Published<ObjP> Pall{&X0->P[0][0]};  // (every group's view, published above)

        const uint32_t mv = (uint32_t)group_ballot<GL>(moved && r < n, gbase);
        bool t0 = false, t1 = false;
        if (r < nr) {
            const RelConst& rc = Hd->rel[r];
            t0 = (((mv >> rc.s) | (mv >> rc.t) | (mv >> rc.as) | (mv >> rc.at)) & 1u) != 0;
        }
        if (r + GL < nr) {
            const RelConst& rc = Hd->rel[r + GL];
            t1 = (((mv >> rc.s) | (mv >> rc.t) | (mv >> rc.as) | (mv >> rc.at)) & 1u) != 0;
        }
        const Staged<double> Sg = Sall.at(g * S_W0);
        if constexpr (BOUND || MH_CHECK) {  // (the exact instance compiles none of it)
            if (bound_b) {
                // The node's bound, this wavefront's share: the VisualBalance products, the moved
                // objects' FocalPoint terms and the touched relationships' terms as fp32 estimates
                // (exact where an estimate cannot vouch for its branch), the rest carried.
                float cph_n = cph, efp_n = efp_c;
                double pw0 = rpw0, an0 = rang0, pw1 = rpw1, an1 = rang1;
                float ea0n = ea0_c, ea1n = ea1_c;
                const ObjP* PGg = Pall.ptr() + g * GL;
                if (moved && r < n) {
                    ObjP p;
                    p.xf = xf;
                    p.yf = yf;
                    p.rotYf = ryf;
                    p.pad = 0.0f;
                    const float fy = rm.fyf - yf, fx = rm.fxf - xf;
                    bool ambo = !(fmaxf(fabsf(fy), fabsf(fx)) >= 0x1p-100f);
                    cph_n = cph_est(atan2_est(fy, fx), p, ambo);
                    efp_n = kDeltaCph;
                    if (ambo) cph_n = __builtin_nanf("");  // (an invalid bound: the node is open)
                }
                auto rel_est = [&](int q, double& pw, double& an, float& ea) __attribute__((always_inline)) {
                    const RelConst& rc = Hd->rel[q];
                    const float4 e0 = Hd->re0[q], e1 = Hd->re1[q];
                    bool amb = false;
                    pw = rel_pw_est(e0, PGg[rc.s], PGg[rc.t], amb);
                    const ObjP as = PGg[rc.as], atp = PGg[rc.at];
                    const float ay = as.yf - atp.yf, ax = as.xf - atp.xf;
                    amb |= !(fmaxf(fabsf(ay), fabsf(ax)) >= 0x1p-100f);
                    // (a pair on one horizontal line, e.g. both clamped to a wall: theta is exactly 0)
                const bool flat = ay == 0.0f && ax > 0.0f;
                an = rel_ang_est(e1, e0.w, atp, flat ? 0.0f : atan2_est(ay, ax), ea, amb, flat);
                    if (amb) pw = __builtin_nan("");  // (an estimate that cannot vouch for its branch:
                                                      // the node is open, its exact terms next batch)
                };
                if (t0) rel_est(r, pw0, an0, ea0n);
                if (t1) rel_est(r + GL, pw1, an1, ea1n);
                BoundTerms bt{};
                bt.k = 8;
                if (r < n) {
                    const float area = __int_as_float(Hd->objs[r].pad);
                    bt.nx = (float)((double)area * sx);  // Kernel.cu:200-201
                    bt.ny = (float)((double)area * sy);
                    bt.anx = fabsf(bt.nx);
                    bt.any = fabsf(bt.ny);
                    bt.fp = -cph_n;
                    bt.afp = fabsf(cph_n);
                    bt.efp = efp_n;
                }
                bt.pw = -(float)(pw0 + pw1);
                bt.ang = -(float)(an0 + an1);
                bt.aang = fabsf(bt.ang);
                bt.eang = ea0n + ea1n;
                bt.pwx = group_ballot<GL>(ea0n > 0.0f || ea1n > 0.0f, gbase) != 0 ? kPwEstU : 0;
                float part[8], sm[8];
                bound_parts(rm, n, c, nr, 0, bt, part);
#pragma unroll
                for (int k = 0; k < 8; ++k) sm[k] = grp8_fsum(part[k]);
                const Staged<float> B{SH->BS[K * hf + g]};
                if (r == 0) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) B.put(k, sm[k]);
                    B.put(11, (float)bt.pwx);
                }
                if (!exact_b) {  // the node's terms and their allowances, for its commit
                    if (r < n) {
                        Sg.put(S_FP + r, -(double)cph_n);
                        stage(Published<float>{X0->EO[g]}).put(r, efp_n);
                    }
                    if (r < nr) {
                        Sg.put(S_PW + r, -pw0);
                        Sg.put(S_ANG + r, -an0);
                    }
                    if (r + GL < nr) {
                        Sg.put(S_PW + r + GL, -pw1);
                        Sg.put(S_ANG + r + GL, -an1);
                    }
                    Sg.put(S_VBX + r, (double)ea0n);
                    Sg.put(S_VBY + r, (double)ea1n);
                }
            }
        }
        SSTAMP(5);
        const Staged<double> SUMst{SH->SUM[par][K * hf + g]};
        if (exact_b) {
            // The exact FocalPoint terms of the group's moved objects and the terms of the
            // relationships they touch (and of the carried terms that are estimates), the rest
            // carried from the incoming state. The group's jobs (relationships first, then
            // objects) are dealt out to its 8 lanes, one double atan2 per lane per pass
            // (Kernel.cu:170-188, 222, 249-253, 271-277).
            const bool fj = r < n && (moved || efp_c != 0.0f);
            const bool t0j = t0 || (r < nr && ea0_c != 0.0f);
            const bool t1j = t1 || (r + GL < nr && ea1_c != 0.0f);
            const uint32_t fm = (uint32_t)group_ballot<GL>(fj, gbase);
            const uint32_t tm = (uint32_t)group_ballot<GL>(t0j, gbase) |
                                ((uint32_t)group_ballot<GL>(t1j, gbase) << GL);
            const int nrt = __builtin_popcount(tm);
            if (r < n) {
                const float area = __int_as_float(Hd->objs[r].pad);
                Sg.put(S_VBX + r, (double)area * sx);  // Kernel.cu:200-201
                Sg.put(S_VBY + r, (double)area * sy);
                if (!fj) Sg.put(S_FP + r, -(double)cph);
            }
            if (r < nr && !t0j) {
                Sg.put(S_PW + r, -rpw0);
                Sg.put(S_ANG + r, -rang0);
            }
            if (r + GL < nr && !t1j) {
                Sg.put(S_PW + r + GL, -rpw1);
                Sg.put(S_ANG + r + GL, -rang1);
            }
            // The 8 nodes' jobs are dealt out to the wavefront's 64 lanes (one pass unless they
            // number more than 64): lane q takes job q of the concatenation, group by group.
            const uint32_t jw = tm | (fm << 16) | ((uint32_t)nrt << 24);  // (group-uniform)
            uint32_t JW[K];
            int JP[K + 1];
            JP[0] = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                JW[k] = (uint32_t)__builtin_amdgcn_readlane((int)jw, k << 3);
                JP[k + 1] = JP[k] + (int)(JW[k] >> 24) + __builtin_popcount((JW[k] >> 16) & 0xffu);
            }
            for (int q0 = 0; q0 < JP[K]; q0 += 64) {  // (wave-uniform trip count)
                const int q = q0 + lane;
                int G = 0, base = 0;
                uint32_t w = JW[0];
#pragma unroll
                for (int k = 1; k < K; ++k) {
                    const bool ge = q >= JP[k];
                    G = ge ? k : G;
                    w = ge ? JW[k] : w;
                    base = ge ? JP[k] : base;
                }
                const int ql = q - base, nrtG = (int)(w >> 24);
                const bool has = q < JP[K], isrel = ql < nrtG;
                const int idx = nth_bit(isrel ? (w & 0xffffu) : ((w >> 16) & 0xffu), isrel ? ql : ql - nrtG);
                const bool rel = has && isrel, foc = has && !isrel;
                const ObjP* PG = Pall.ptr() + G * GL;
                const RelConst& rc = Hd->rel[rel ? idx : 0];
                const ObjP qo = PG[foc ? idx : 0];
                double ay = 0.0, ax = 1.0, pw = 0.0;
                float ti = 0.0f;
                if (rel) pw = rel_pair(rc, PG, ay, ax, ti);
                if (foc) {
                    ay = (double)(rm.fyf - qo.yf);
                    ax = (double)(rm.fxf - qo.xf);
                }
                const double at = atan2_ool(ay, ax);
                const Staged<double> SG = Sall.at(G * S_W0);
                if (rel) {
                    SG.put(S_PW + idx, -pw);
                    SG.put(S_ANG + idx, -rel_angle(rc, at, ti));
                }
                if (foc) {  // focal_cos with the atan2 above (atan2_f32 rounds it once)
                    const float b = (float)at - qo.rotYf;
                    SG.put(S_FP + idx, -(double)cos_f32((float)((double)b + kHalfPI)));
                }
            }
            const Published<double> Sv = publish(Sall);
            SSTAMP(3);
            // The eight ordered sums: lane r of each group replays stream r (float sums round
            // every partial sum to float; a double-rounded float add equals the float add, 53 >=
            // 2*24+2), in the wavefront that built it (the list wavefront: 3, 4, 5); the workgroup
            // barrier hands every node's to both chain wavefronts. The buffer alternates by batch.
            if (r <= 2 || r >= 6) {
                int base = S_VBX, len = n;
                bool rnd = true;
                switch (r) {
                    case 0: base = S_VBX; len = n; rnd = true; break;
                    case 1: base = S_VBY; len = n; rnd = true; break;
                    case 2: base = S_FP; len = n; rnd = false; break;
                    case 6: base = S_PW; len = nr; rnd = false; break;
                    default: base = S_ANG; len = nr; rnd = false; break;
                }
                const double* src = Sv.ptr() + g * S_W0 + base;
                double acc = 0.0;
                for (int l = 0; l < len; ++l) {
                    const double s = acc + src[l];
                    acc = rnd ? (double)(float)s : s;
                }
                SUMst.put(r, acc);
            }
        }
        SSTAMP(4);
        const Published<double> SUMv = publish_workgroup(SUMst);
        // (every half's streams and bound sums were published by its wavefronts before the same
        // barrier; they are next rewritten after the next batch's views barrier)
        auto streams_of = [&](int h) __attribute__((always_inline)) {
            return Published<double>{&X0of(h)->S[0][0]};
        };
        const Published<float> BSv{&SH->BS[0][0]};
        par ^= 1;
        SSTAMP(6);
        // Node `lane` (lanes 0 .. NN-1; the others repeat node 0).
        const int nd = lane < NN ? lane : 0;
        // Accept (Kernel.cu:706-713) at every node: its step's uniform against its current
        // total (the node whose configuration it started from, or the batch's incoming total).
        const float u_dep = shfl_f(r_u, tr.dep < 64 ? tr.dep : 0);  // (record dep's uniform)
        const float u_n = tr.dep < kb ? u_dep : 1.0f;
        const int cpar_l = tr.cpar == kNone ? 0 : tr.cpar;
        float sc[8];
        uint64_t ab = 0ull, ob = 0ull;  // accepted nodes; nodes the bound leaves open
        float st_lo = 0.0f, st_hi = 0.0f;  // (bound batches) each node's total's interval
        if (exact_b) {
            // Costs(), Kernel.cu:518-549 (OffLimits never enters a step, :547)
            const double* sm = SUMv.ptr() + (nd - (K * hf + g)) * 8;  // (SUM[par][nd])
            const float nx = (float)sm[0], ny = (float)sm[1];
            const double fpd = sm[2];
            const float symf = (float)sm[3], clf = (float)sm[4], saf = (float)sm[5];
            const float pw = (float)(sm[6] * sm[7]);
            const float vb = (float)(-1.0 * distance_f(nx / rm.denom, ny / rm.denom, rm.cxf, rm.cyf));
            sc[1] = rm.w_pw * pw;
            sc[2] = rm.w_vb * vb;
            sc[3] = rm.w_fp * (float)fpd;
            sc[4] = rm.w_sym * symf;
            sc[6] = rm.w_ol * 0.0f;
            sc[5] = rm.w_cl * clf;
            sc[7] = rm.w_sa * saf;
            float t = sc[1] + sc[2];
            t = t + sc[3];
            t = t + sc[4];
            t = t + sc[5];
            t = t + sc[7];
            sc[0] = t;
            const float cp_tot = shfl_f(sc[0], cpar_l);
            // (a refresh: the root's current total is node NN - 1's, the incoming configuration's)
            const float cur0 = refresh ? readlane_f(sc[0], NN - 1) : cur[0];
            const float cur_n = tr.cpar == kNone ? cur0 : cp_tot;
            const bool acc_n = lane < NN && tr.dep < kb && !(refresh && lane == NN - 1) &&
                               accept_u(u_n, kBeta * ((double)sc[0] - (double)cur_n));
            ab = __ballot(acc_n);
        }
        if constexpr (BOUND || MH_CHECK) {  // (the exact instance compiles none of it)
            if (bound_b) {
                // the node's bound: its chain and list wavefronts' sums, composed (bound_te; the
                // decision's arithmetic on the current total added per node, as bound_compose does)
                const float* bs = BSv.ptr() + nd * kBS;
                float sum[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) sum[k] = bs[k] + (k >= 4 && k <= 6 ? bs[8 + (k - 4)] : 0.0f);
                BoundTerms unused{};
                float e0;
                const float t = bound_te<false>(rm, n, nr, 8, (int)bs[11], sum, unused, CostIv{0.0f, 0.0f},
                                                a.bound_slack, e0);
                st_lo = t - 1.5f * e0;
                st_hi = t + 1.5f * e0;
                const float plo = shfl_f(st_lo, cpar_l), phi = shfl_f(st_hi, cpar_l);
                CostIv cur_n = tr.cpar == kNone ? cur_iv : CostIv{plo, phi};
#if MH_CHECK
                // (check builds: against the exact current totals the exact decisions use)
                {
                    const float pcx = shfl_f(sc[0], cpar_l);  // (every lane: an inactive source reads 0)
                    const float cx0 = tr.cpar == kNone ? cur[0] : pcx;
                    cur_n = CostIv{cx0, cx0};
                }
#endif
                const float e = e0 + a.bound_slack * (3.0f * 0x1p-24f) *
                                         fmaxf(fabsf(cur_n.lo), fabsf(cur_n.hi));
                CostIv star;
                const int d = bound_vs(t, e, u_n, cur_n, star);
                const bool live = lane < NN && tr.dep < kb;
#if MH_CHECK
                if (live) {
                    const bool acc_x = ((ab >> lane) & 1ull) != 0;
                    MH_CK(st_lo != st_lo || (sc[0] >= st_lo && sc[0] <= st_hi), 22, __float_as_uint(sc[0]),
                          __float_as_uint(st_hi - st_lo));
                    MH_CK(d != BOUND_REJECT || !acc_x, 20, __float_as_uint(sc[0]), __float_as_uint(t));
                    MH_CK(d != BOUND_ACCEPT || acc_x, 21, __float_as_uint(sc[0]), __float_as_uint(t));
                    if ((d == BOUND_REJECT && acc_x) || (d == BOUND_ACCEPT && !acc_x)) {
                        if (atomicCAS(&g_spec_ck[0], 0u, 1u) == 0u) {  // (the first one's inputs)
                            g_spec_ck[1] = __float_as_uint(sc[0]);
                            g_spec_ck[2] = __float_as_uint(t);
                            g_spec_ck[3] = __float_as_uint(e);
                            g_spec_ck[4] = __float_as_uint(cur_n.lo);
                            g_spec_ck[5] = __float_as_uint(u_n);
                            g_spec_ck[6] = (unsigned)d | ((unsigned)lane << 8) | ((unsigned)tr.dep << 16);
                            g_spec_ck[7] = (unsigned)tr.cpar | ((unsigned)kb << 8) | ((unsigned)H << 16);
                            g_spec_ck[8] = __float_as_uint(cur[0]);
                            g_spec_ck[9] = (unsigned)done;
                            g_spec_ck[10] = __float_as_uint(e0);
                            g_spec_ck[11] = (unsigned)hf;
                        }
                    }
                    mh_count_decision(d, true);
                    atomicAdd(&g_check[5], 1u);
                }
#else
                ab = __ballot(live && d == BOUND_ACCEPT);
                ob = __ballot(live && d == BOUND_OPEN);
#endif
            }
        }
        // The realised path from the root: its nodes' steps commit; the configuration after
        // them is the last accepted node's (or the incoming one). A node the bound leaves open
        // ends the path before its step, which the next batch evaluates exactly.
        int node = 0, steps = 0, last = kNone, nacc = 0;
        unsigned int acc_steps = 0;
#pragma unroll
        for (int d = 0; d < NN; ++d) {
            if (node == kNone || (refresh && node == NN - 1) || d >= kb) break;
            if ((ob >> node) & 1ull) {
                exact_next = true;
                break;
            }
            ++steps;
            const bool an = ((ab >> node) & 1ull) != 0;
            if (an) {
                last = node;
                ++nacc;
                acc_steps |= 1u << d;
            }
            node = __builtin_amdgcn_readlane(an ? tr.cha : tr.chr, node);
        }
        if constexpr (BOUND && !MH_CHECK) {
            if (exact_b) {
                if (exact_next) exact_next = false;
                else if (exact_run > 0) --exact_run;
            } else if (exact_next) {  // this bound batch stopped at an open node
                backoff = since_open < 4 ? min(2 * backoff, 64) : 1;
                exact_run = backoff - 1;
                since_open = 0;
            } else {
                ++since_open;
            }
        }
        if (refresh) {
            // node NN - 1 evaluated the incoming configuration: its exact costs and terms are the
            // current ones (until a committed node's replace them below)
            const double* sl = streams_of((NN - 1) / K).ptr() + ((NN - 1) % K) * S_W0;
            if (r < n) cph = (float)(-sl[S_FP + r]);
            if (r < nr) {
                rpw0 = -sl[S_PW + r];
                rang0 = -sl[S_ANG + r];
            }
            if (r + GL < nr) {
                rpw1 = -sl[S_PW + r + GL];
                rang1 = -sl[S_ANG + r + GL];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) cur[k] = readlane_f(sc[k], NN - 1);
            cur_iv = CostIv{cur[0], cur[0]};
            cur_exact = true;
            efp_c = ea0_c = ea1_c = 0.0f;
        }
        if (last != kNone) {
            const int lh = last / K, lg = last % K;
            if (H == 1 || lh == hf) {  // this wavefront's node: its group holds the configuration
                const int src = (lg << 3) + r;
                cx = shfl_d(sx, src);
                cy = shfl_d(sy, src);
                cry = shfl_d(sry, src);
            } else if constexpr (H > 1) {  // the other half's: the path's proposals again
                bool mv2 = false;
                apply(cx, cy, cry, mv2, steps, [&](int i) __attribute__((always_inline)) {
                    return ((acc_steps >> i) & 1u) != 0;
                });
            }
            const double* sl = streams_of(lh).ptr() + lg * S_W0;
            if (r < n) cph = (float)(-sl[S_FP + r]);
            if (r < nr) {
                rpw0 = -sl[S_PW + r];
                rang0 = -sl[S_ANG + r];
            }
            if (r + GL < nr) {
                rpw1 = -sl[S_PW + r + GL];
                rang1 = -sl[S_ANG + r + GL];
            }
            if (exact_b) {  // (every term of an exact batch's node is exact)
#pragma unroll
                for (int k = 0; k < 8; ++k) cur[k] = readlane_f(sc[k], last);
                cur_iv = CostIv{cur[0], cur[0]};
                cur_exact = true;
                efp_c = ea0_c = ea1_c = 0.0f;
            } else {
                cur_iv = CostIv{readlane_f(st_lo, last), readlane_f(st_hi, last)};
                cur_exact = false;
                efp_c = r < n ? X0of(lh)->EO[lg][r] : 0.0f;
                ea0_c = (float)sl[S_VBX + r];
                ea1_c = (float)sl[S_VBY + r];
            }
            accepted += (unsigned int)nacc;
            // An accepted swap also exchanges z, rotX and rotZ (:675-700), object 1's values
            // through float temporaries, in step order (a later swap sees an earlier one's).
            for (int d = 0; d < steps; ++d) {
                if (!((acc_steps >> d) & 1u)) continue;
                const int qc = __builtin_amdgcn_readlane(r_code, d);
                const int q1 = rec_k1(qc), q2 = rec_k2(qc);
                if (rec_mode(qc) == 2 && q1 >= 0) {
                    const int ia = gbase + q1, ib = gbase + q2;
                    const double az = shfl_d(cz, ia), arx = shfl_d(crx, ia), arz = shfl_d(crz, ia);
                    const double bz = shfl_d(cz, ib), brx = shfl_d(crx, ib), brz = shfl_d(crz, ib);
                    if (r == q2) {
                        cz = (double)(float)az;
                        crx = (double)(float)arx;
                        crz = (double)(float)arz;
                    } else if (r == q1) {
                        cz = bz;
                        crx = brx;
                        crz = brz;
                    }
                }
            }
        }
#if MH_SPEC_DEBUG
        if (chain == 0 && lead && lane == 0) {  // [done, kb, cons, prod_seen, last, steps, cur0, nacc]
            const unsigned int base = g_spec_dbg_n;
            if (base + 8 < (1u << 16)) {
                g_spec_dbg[base + 0] = (unsigned)done;
                g_spec_dbg[base + 1] = (unsigned)kb;
                g_spec_dbg[base + 2] = cons;
                g_spec_dbg[base + 3] = prod_seen;
                g_spec_dbg[base + 4] = (unsigned)last;
                g_spec_dbg[base + 5] = (unsigned)steps;
                g_spec_dbg[base + 6] = __float_as_uint(cur_iv.lo);
                g_spec_dbg[base + 7] = (unsigned)nacc | (exact_b ? 0x100u : 0u) | (refresh ? 0x200u : 0u);
                g_spec_dbg_n = base + 8;
            }
        }
#endif
        // The stream's state after the committed steps: what the last of them leaves (read
        // before the count is published: wave 1 may then reuse the slot).
        if (steps > 0) {
            const StepRec& q = rec(cons + (unsigned int)(steps - 1));
            end_pos = ((uint64_t)q.next_hi << 32) | q.next_lo;
            end_h = rec_h(q.code);
            end_bv = q.bv;
        }
        cons += (unsigned int)steps;
        done += steps;
        if (lead && lane == 0) CONS.put(0, cons);  // (wave 1 reads it between the next two barriers)
        SSTAMP(7);
#if MH_STAMPS
        cyc[14] += 1;
        cyc[15] += (unsigned long long)steps;
        cyc[13] += exact_b ? 1 : 0;
        cyc[12] += refresh ? 1 : 0;
#endif
    }
#if MH_STAMPS
    {
        unsigned long long rt1;
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rt1) :: "memory");
        cyc[8] = t_last - t_first;  // shader cycles of the loop
        cyc[9] = rt1 - rt0;         // 100 MHz ticks of the same span
        if (lead && lane == 0 && chain < 16384) {
            const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_ID
            const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // XCC_ID
            g_spec_place[6 * chain + 0] = rt0;
            g_spec_place[6 * chain + 1] = rt1;
            g_spec_place[6 * chain + 2] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
            g_spec_place[6 * chain + 3] = cyc[14];
            g_spec_place[6 * chain + 4] = cyc[13];
            g_spec_place[6 * chain + 5] = cyc[12];
        }
    }
    if (lead && lane == 0)  // (wave 0's timeline; its wait for wave 1 lands in "ordered sums")
        for (int k = 0; k < 16; ++k) atomicAdd(&g_spec_cycles[k], cyc[k]);
#endif

    if (lead && lane < n) {
        st[F_X * n + r] = cx;
        st[F_Y * n + r] = cy;
        st[F_RY * n + r] = cry;
        st[F_Z * n + r] = cz;
        st[F_RX * n + r] = crx;
        st[F_RZ * n + r] = crz;
    }
    if (lead && lane == 0) {
        ChainMeta m = m0;
        m.accepted = m0.accepted + accepted;
        m.draws = end_pos;
        m.bm_has = end_h;
        m.bm_val = end_bv;
#pragma unroll
        for (int k = 0; k < 8; ++k) m.costs[k] = cur[k];
        a.meta[chain] = m;
    }
}

}  // namespace

#if MH_SPEC_DEBUG
extern "C" __attribute__((visibility("default"))) int mh_debug_spec(unsigned int* out, int cap) {
    unsigned int n = 0;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_spec_dbg_n), sizeof(n)) != hipSuccess) return -1;
    if ((int)n > cap) n = (unsigned)cap;
    if (n && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_spec_dbg), sizeof(unsigned) * n) != hipSuccess) return -1;
    const unsigned int zero = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_spec_dbg_n), &zero, sizeof(zero));
    return (int)n;
}
#endif

#if MH_STAMPS
extern "C" __attribute__((visibility("default"))) int mh_debug_spec_place(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_spec_place), sizeof(unsigned long long) * 6 * 16384) ==
                   hipSuccess ? 0 : -1;
}
extern "C" __attribute__((visibility("default"))) int mh_debug_spec_simd(unsigned int* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_spec_simd), sizeof(unsigned int) * 4 * 16384) ==
                   hipSuccess ? 0 : -1;
}
extern "C" __attribute__((visibility("default"))) int mh_debug_spec_cycles(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_spec_cycles), sizeof(unsigned long long) * 16) != hipSuccess)
        return -1;
    unsigned long long zero[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_spec_cycles), zero, sizeof(zero));
    return 0;
}
#endif

// The kernel instance: H = 2 (16 nodes, four wavefronts per chain) or 1 (8 nodes, two).
size_t spec_lds_bytes(int halves) { return (size_t)(halves >= 2 ? spec_bytes<2>() : spec_bytes<1>()); }

// Chains per workgroup (one: its wavefronts share the chain), and wavefronts per chain.
int spec_waves() { return 1; }
int spec_waves_per_chain(int halves) { return 2 * (halves >= 2 ? 2 : 1); }

// Whether the speculative kernel serves a room: at most GL objects, RMAX relationships.
bool spec_fits(int n, int c, int r) { return n >= 1 && n <= GL && c <= GL && r <= RMAX; }

template <int H, bool B>
int spec_blocks_of() {
    int blocks = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, mh_spec_kernel<H, B>,
                                                                       128 * H, spec_lds_bytes(H));
    return e == hipSuccess ? blocks : 0;
}

int spec_blocks_per_cu(int halves, bool bound) {
    if (halves >= 2) return bound ? spec_blocks_of<2, true>() : spec_blocks_of<2, false>();
    return bound ? spec_blocks_of<1, true>() : spec_blocks_of<1, false>();
}

// The instance: halves, and decisions on the bound (a.spec_bound) or on exact costs alone.
template <int H, bool B>
void launch_spec_of(const LaunchArgs& a, hipStream_t s) {
    hipLaunchKernelGGL((mh_spec_kernel<H, B>), dim3((unsigned)a.n_chains), dim3(128 * H),
                       spec_lds_bytes(H), s, a);  // (one chain per workgroup)
}

hipError_t launch_spec(const LaunchArgs& a, int halves, hipStream_t s) {
    if (a.n_chains <= 0) return hipSuccess;
    if (halves >= 2) {
        if (a.spec_bound) launch_spec_of<2, true>(a, s);
        else launch_spec_of<2, false>(a, s);
    } else {
        if (a.spec_bound) launch_spec_of<1, true>(a, s);
        else launch_spec_of<1, false>(a, s);
    }
    return hipGetLastError();
}

}  // namespace mh

#if MH_CHECK
extern "C" __attribute__((visibility("default"))) int mh_debug_spec_ck(unsigned int* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_spec_ck), sizeof(unsigned int) * 12) == hipSuccess ? 0 : -1;
}
extern "C" __attribute__((visibility("default"))) int mh_debug_check_spec(unsigned int* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_check), sizeof(unsigned int) * 8) == hipSuccess ? 0 : -1;
}
extern "C" __attribute__((visibility("default"))) int mh_debug_decisions_spec(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_decide), sizeof(unsigned long long) * 4) ==
                   hipSuccess ? 0 : -1;
}
#endif
