// mh_device.h -- POD layouts shared by the host library (mh_abi.cpp) and the HIP kernels
// (mh_chain.hip). Everything here is derived on the host from the KernelWrapper inputs
// (Kernel.cu:873) so the device never re-derives per-room constants.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define MH_HD __host__ __device__
#else
#define MH_HD
#endif

namespace mh {

// Reference constants, Kernel.cu:31-39 (PI is 3.1416, not M_PI).
constexpr double kPI = 3.1416;
constexpr double kTwoPI = 2 * 3.1416;
constexpr double kHalfPI = 3.1416 / 2.0;
constexpr double kSigmaT = 15.0 / 90.0 * 3.1416;
constexpr double kBeta = 2.0;

// Axis-aligned box of a four-vertex rectangle as minValue/maxValue (Kernel.cu:366-401) see it,
// reduced on the host: for a translation (tx, ty) the box is
//   min.x = min(v0x, rn_d(xmin1 + tx))   (the first vertex enters untranslated, Kernel.cu:371)
//   max.x = rn_d(xmax + tx), min.y = rn_d(ymin + ty), max.y = rn_d(ymax + ty)
// and is then rounded to float (calculateIntersectionArea's fmaxf/fminf, Kernel.cu:325-328).
// Rounding is monotone, so the running min/max of the reference equals these closed forms.
struct RectShape {
    float v0x;  // (float) of vertex 0's x
    int pad;
    double xmin1;  // min over vertices 1..3 of x
    double xmax;   // max over vertices 0..3 of x
    double ymin;   // min over vertices 0..3 of y
    double ymax;
};

struct ObjConst {   // one per object
    RectShape off;  // its off-limits rectangle (offlimits[j].point1Index)
    float area;     // (float)(length * width), VisualBalanceCosts Kernel.cu:199
    int frozen;
};

struct ClrConst {   // one per clearance
    RectShape shape;
    int src;        // clearances[i].SourceIndex
    int pad;
};

struct RelConst {   // relationship i: rss[i] and rsa[i] (sized by nRelationships, Kernel.cu:880,885)
    double start, end;  // rss[i].TargetRange
    double amin, amax;  // rsa[i].angleMin / angleMax
    int s, t;           // rss[i] Source / Target
    int as, at;         // rsa[i] Source / Target
    double norm_w;      // (2PI - (amax + (2PI - amin))) / 2, Kernel.cu:247 (wrapped range)
    double norm_n;      // (2PI - (amax - amin)) / 2, Kernel.cu:255 (plain range)
};

// Allowances of the rejection bound's fp32 estimates (derivation: mh_common.h, above atan2_est).
constexpr float kDeltaCph = 0x1p-17f;
constexpr float kDeltaTh = 0x1p-17f;
constexpr int kPwEstU = 20;

// The fp32 constants of relationship i's estimates (two float4 per relationship; the
// full-evaluation kernel stages them in LDS, the incremental kernel reads them from HBM with the
// records a move touches -- built on the host, LaunchArgs::rele):
//   e0 = {(float)start, (float)end, 1 / start, the angle allowance's constant part}
//   e1 = {(float)amin, (float)amax, 1 / norm of the range (wrapped or plain), flags}
// flags: bit 0 the range wraps (amin > amax, Kernel.cu:245); bit 1 no estimate (the term is
// always evaluated exactly): a degenerate normaliser (|norm| < 1e-3), |amin| or |amax| >= 64, or
// a non-finite constant. The angle allowance: theta within kDeltaTh, amin / amax rounded to
// float (U |a| <= kDeltaTh / 2 for |a| < 64) and the subtraction, min and product roundings (3 U
// |v|): 2 kDeltaTh |1 / norm| + 4 U |v| covers them; e0.w is the first part rounded up.
enum { RE_WRAP = 1, RE_EXACT = 2 };
template <class F4>
inline MH_HD void rel_est_consts(const RelConst& rc, F4& e0, F4& e1) {
    const bool wrap = rc.amin > rc.amax;
    const double norm = wrap ? rc.norm_w : rc.norm_n;
    const double an = norm < 0 ? -norm : norm;
    const double a0 = rc.amin < 0 ? -rc.amin : rc.amin, a1 = rc.amax < 0 ? -rc.amax : rc.amax;
    const double s0 = rc.start < 0 ? -rc.start : rc.start, s1 = rc.end < 0 ? -rc.end : rc.end;
    const bool ok = an >= 1e-3 && a0 < 64.0 && a1 < 64.0 && s0 < 1e30 && s1 < 1e30 &&
                    rc.start != 0.0;
    e0.x = (float)rc.start;
    e0.y = (float)rc.end;
    e0.z = ok ? (float)(1.0 / rc.start) : 0.0f;
    e0.w = ok ? (float)(2.0 * (double)kDeltaTh / an * (1.0 + 0x1p-20)) : 0.0f;
    e1.x = (float)rc.amin;
    e1.y = (float)rc.amax;
    e1.z = ok ? (float)(1.0 / norm) : 0.0f;
    e1.w = __builtin_bit_cast(float, (wrap ? RE_WRAP : 0) | (ok ? 0 : RE_EXACT));
}

// Scalars of one room, passed by value as a kernel argument.
struct DevRoom {
    int n, c, r, pad0;
    float w_pw, w_vb, w_fp, w_sym, w_ol, w_cl, w_sa;
    float fxf, fyf;    // (float)focalX, (float)focalY: phi() arguments, Kernel.cu:271
    float ux, uy;      // (float)cos(focalRot), (float)sin(focalRot), Kernel.cu:290-291
    float cxf, cyf;    // (float)(centroidX / 2), (float)(centroidY / 2), Kernel.cu:206
    float denom;       // sequential float sum of areas, Kernel.cu:202
    float sx, sy;      // proposal std devs width/16, height/16, Kernel.cu:587-591
    float inv_denom;   // 1 / denom rounded to float (the rejection bound only)
    double along_f;        // focalX*ux + focalY*uy, Kernel.cu:292
    double two_focal_rot;  // 2 * focalRot, Kernel.cu:297
    double rmin_x, rmin_y, rmax_x, rmax_y;  // room box for the translate clamp, Kernel.cu:613-630
    float comp[4][4];      // complement rectangles (minx, miny, maxx, maxy) as floats, Kernel.cu:343-364
};

// Per-chain persistent state besides the poses.
struct ChainMeta {
    uint64_t draws;     // Philox outputs consumed so far (rocrand offset)
    uint64_t accepted;  // accepted proposals so far
    int bm_has;         // Box-Muller cache flag
    float bm_val;       // cached second normal
    float costs[8];     // resultCosts of the current state
    float best_total;   // best-of-chain tracking: totalCosts of the saved best configuration
    int rung;           // parallel tempering: this chain's temperature index (0 = BETA)
};
static_assert(sizeof(ChainMeta) == 64, "ChainMeta");

// Pose layout in HBM: chain-major, six SoA rows of N doubles.
// x, y, rotY enter the costs; z, rotX, rotZ (contiguous, F_Z..F_RZ) never do.
enum { F_X = 0, F_Y = 1, F_RY = 2, F_Z = 3, F_RX = 4, F_RZ = 5, F_COUNT = 6 };

// Best-of-chain tracking (the reference's commented-out cfgBest/bestCosts, Kernel.cu:779-782,
// 808-816, 835-860): 0 off (the reference as shipped: output = final current state),
// 1 = lowest totalCosts (the commented code's `starCosts->totalCosts < bestCosts->totalCosts`),
// 2 = highest totalCosts (the direction Accept climbs, Kernel.cu:706-713).
enum { TRACK_OFF = 0, TRACK_LOWEST = 1, TRACK_HIGHEST = 2 };

__device__ __forceinline__ bool best_improves(int track, float star, float best) {
    return track == TRACK_LOWEST ? star < best : star > best;  // NaN never improves
}

// Saves the proposed configuration (cfgStar, Kernel.cu:810-811) of one chain to its best
// slot `dst` ([6][N] like the chain state). Lane r of the chain's L lanes writes objects
// r, r+L, ... x, y, rotY come from LDS; z, rotX, rotZ live in HBM (`ch.zrr`) and are swapped
// there only on accept, so a pending swap (aux->swap_a/b >= 0) is applied here as
// commit_swap_zrr would: ka takes kb's values, kb takes ka's rounded to float.
template <class Ptrs>
__device__ __forceinline__ void save_best(const Ptrs& ch, double* dst, int n, int r, int L) {
    const int ka = ch.aux->swap_a, kb = ch.aux->swap_b;
    for (int i = r; i < n; i += L) {
        dst[F_X * n + i] = ch.X[i];
        dst[F_Y * n + i] = ch.Y[i];
        dst[F_RY * n + i] = ch.RY[i];
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

// Per-chain scalars of the full-evaluation kernel (mh_chain.hip ChainAux), bytes.
#if defined(MH_STAMPS) && MH_STAMPS
constexpr int kChainAuxBytes = 272;
#else
constexpr int kChainAuxBytes = 176;
#endif

// LDS carve-up of the full-evaluation kernel. One workgroup = WAVES waves; each wave holds
// G = 64/L chains. The room tables are kept as 40-byte RectShape records: an object's
// off-limits rectangle with its area in .pad, a clearance's rectangle with its source in .pad.
struct ChainLds {
    int hdr;     // bytes of the per-workgroup header: room tables + frozen flags
    int h_obj;   // RectShape[N] within the header (pad = area bits)
    int h_clr;   // RectShape[C] (pad = source object)
    int h_rel;   // RelConst[R]
    int h_rix;   // uint2[R] the relationships' objects {s | t << 16, as | at << 16}: the step's
                 // per-lane "does the move touch relationship i" test reads these 8-byte words
                 // (the 64-byte RelConst stride put all 32 lanes on two banks)
    int h_re;    // float4[2][R] the relationships' fp32 estimate constants (rel_est_consts)
    int h_frz;   // unsigned char[N + 1] frozen flags (index N counts as frozen)
    int h_room;  // DevRoom copy (read by the out-of-line cost evaluation)
    int P;       // ObjP[N]   {float xf, yf, rotYf, pad} (the double x, y, rotY live in the
                 // owner lanes' registers; z, rotX, rotZ never enter a cost: they stay in HBM)
    int OFF;     // float4[N] off-limits boxes (final / evaluation passes only; -1 in the step)
    int CLA;     // float4[C] clearance boxes at their source objects
    int NZ;      // uint64[2][C] non-zero Clearance pairs per clearance row (bit j: object j),
                 // current / proposed (incremental pairs, one object per lane)
    int PRE;     // int[C] row prefix counts of the proposed rows
    int AUX;     // ChainAux: proposal backups and the current costs
    int PX, PY;    // double[N4] per-object VisualBalance products (N4 = round4(N), zero past N)
    int CPHF, RMXF;  // float[N4] per-object -cos(phi) and -row max
    int LCL;     // float[2L]    compacted non-zero Clearance terms
    int LPW, LANG;  // double[lst_r] compacted non-zero PairWise / Angle terms
    int lst_r;   // round4(min(L, max(R, 1)))
    int N4;
    int stride;  // bytes per chain
};

inline MH_HD int round16(int v) { return (v + 15) & ~15; }

// Next 16-byte-aligned offset >= o whose 16-byte bank slot (offset / 16 mod 16) is not in
// *used; marks it. Arrays that the lanes of one wave read with the same instruction at the
// same index then start on different LDS banks (bank = address / 4 mod 64).
inline MH_HD int bank_place(int o, unsigned* used) {
    o = round16(o);
    for (int k = 0; k < 16 && ((*used >> ((o >> 4) & 15)) & 1u); ++k) o += 16;
    *used |= 1u << ((o >> 4) & 15);
    return o;
}

// LDS carve-up of the incremental step kernel (mh_delta.hip): per-workgroup room tables (object
// and clearance rectangles, the relationships' objects as 16-bit pairs {s, t, as, at}; the relationship
// records themselves stay in HBM) plus three replay streams (areas, ones, zeros), then per
// chain the configuration and every cached quantity a proposal changes only locally that other
// lanes read (rotY and the symmetry rows live in the owner lanes' registers). The replay reads
// each ordered sum as a stream of NP = round4(N + 1) entries, zero past its end.
struct DeltaLds {
    int hdr, h_obj, h_clr, h_rel, h_frz, h_room;
    int h_area, h_ones, h_zero;  // float[DL] areas, float[DL] ones, double[DL] zeros then 4
                                 // float zeros (each typed as the replay reads it)
    int NP;
    int NR;         // relationship stream length round4(max(R, 1))
    int DL;         // dense replay length max(NP, NR)
    int X, Y;       // double[NP] (zero past N)
    int BOX;        // float4[NP] object off-limits boxes at the current poses (zero past N)
    int RYF;        // float[NP] (float)rotY
    int CPH;        // float[NP] -cos(phi), the FocalPoint terms (zero past N)
    int NMX;        // float[NP] -(row max) of the proposed symmetry rows (the replay's stream)
    int CLA;        // float4[C - 64] boxes of clearances 64.. at their source objects (the first
                    // 64 live in the owner lanes' registers)
    int NZ;         // uint64[C - 64][W] non-zero Clearance pairs of clearances 64.. (row =
                    // clearance, bit = object; rows 0..63 live in the owner lanes' registers)
    int SAM, SAMB;  // uint32[SW] non-zero SurfaceArea entries (C clearances then N objects), backup
    int RPW, RANG;  // double[NR] negated PairWise / PairWiseAngle terms (zero past R)
    int LCL, LSA;   // float[cap] compacted negated Clearance / SurfaceArea terms (zero filled
                    // to round4(count))
    int AUX;        // per-chain scalars (backups, current costs)
    int W, SW;      // words per NZ row (the kernel's object slots), SAM words
    int cap_cl, cap_sa;
    int stride;     // bytes per chain
};

constexpr int kDeltaAuxBytes = 80;  // mh_delta.hip DeltaAux: two undo records, the swap

inline MH_HD DeltaLds make_delta_layout(int n, int c, int r) {
    DeltaLds l;
    const int np = (n + 1 + 3) & ~3;
    l.NP = np;
    int h = 0;
    l.h_obj = h;  h += round16((int)sizeof(RectShape) * n);
    l.h_clr = h;  h += round16((int)sizeof(RectShape) * (c > 0 ? c : 1));
    l.h_rel = h;  h += round16(8 * (r > 0 ? r : 1));
    l.h_frz = h;  h += round16(n + 1);
    l.h_room = h; h += round16((int)sizeof(DevRoom));
    l.NR = ((r > 1 ? r : 1) + 3) & ~3;
    l.DL = np > l.NR ? np : l.NR;
    l.h_area = h; h += round16(4 * l.DL);
    l.h_ones = h; h += round16(4 * l.DL);
    l.h_zero = h; h += round16(8 * l.DL) + 16;
    l.hdr = h;
    l.W = n <= 64 ? 1 : n <= 128 ? 2 : n <= 256 ? 4 : 8;  // the kernel instance's object slots
    l.SW = (c + n + 31) / 32;
    // Clearance list capacity: the non-zero pairs of a sampled room run to ~4 per object at
    // N = 128..256 (tools/stamps.py counts build); longer lists are summed in windows.
    l.cap_cl = 4 * np < 32 ? 32 : 4 * np;
    // SurfaceArea list: a few dozen non-zero terms in sampled rooms (18 at N = 256), so NP / 4.
    l.cap_sa = np / 4 < 32 ? 32 : ((np / 4 + 3) & ~3);
    const int nrp = l.NR;
    int o = 0;
    l.X = o;    o += 8 * np;
    l.Y = o;    o += 8 * np;
    l.BOX = o;  o += 16 * np;
    l.RYF = o;  o += 4 * np;
    l.CPH = o;  o += 4 * np;
    l.NMX = o;  o += round16(4 * np);
    l.CLA = o;  o += 16 * (c > 64 ? c - 64 : 1);  // clearances 64.. (the first 64: registers)
    l.NZ = o;   o += 8 * l.W * (c > 64 ? c - 64 : 1);  // rows 64..: the first 64 are registers
    l.RPW = o;  o += 8 * nrp;
    l.RANG = o; o += round16(8 * nrp);
    l.SAM = o;  o += 4 * l.SW;
    l.SAMB = o; o += round16(4 * l.SW);
    l.LCL = o;  o += 4 * l.cap_cl;
    l.LSA = o;  o += round16(4 * l.cap_sa);
    l.AUX = o;  o += kDeltaAuxBytes;
    o = round16(o);
    if ((o & 255) == 0) o += 16;  // spread the chains' arrays over the LDS banks
    l.stride = o;
    return l;
}

// Objects per lane of the full-evaluation kernel instance that serves npl (mh_chain.hip launch()).
inline MH_HD constexpr int npl_instance(int npl) { return npl <= 1 ? 1 : npl <= 2 ? 2 : npl <= 4 ? 4 : 8; }

inline MH_HD constexpr int round16c(int v) { return (v + 15) & ~15; }

inline MH_HD constexpr int bank_place_c(int o, unsigned& used) {
    o = round16c(o);
    for (int k = 0; k < 16 && ((used >> ((o >> 4) & 15)) & 1u); ++k) o += 16;
    used |= 1u << ((o >> 4) & 15);
    return o;
}

// The part of the full-evaluation kernel's LDS layout that depends only on the kernel instance
// (L lanes, NPL objects per lane: capacity NC = L * NPL objects). The kernel addresses these
// arrays at compile-time offsets (immediate ds_read/ds_write offsets, no SGPRs); the host sizes
// the workgroup with the same function. Header: DevRoom, object shapes, frozen flags, then the
// clearance shapes; the relationship table follows at a run-time offset.
struct FixedLds {
    int h_room, h_obj, h_frz, h_zero, h_clr;            // workgroup header (h_zero: 4 zero doubles)
    int P, AUX, PX, PY, CPHF, RMXF, LCL, RNG, end;  // per chain (RNG: L = 64 only)
};

inline MH_HD constexpr FixedLds fixed_lds(int L, int NPL) {
    const int NC = L * NPL;
    FixedLds f{};
    f.h_room = 0;
    f.h_obj = round16c((int)sizeof(DevRoom));
    f.h_frz = f.h_obj + round16c((int)sizeof(RectShape) * NC);
    f.h_zero = f.h_frz + round16c(NC + 1);
    f.h_clr = f.h_zero + 32;
    int o = 0;
    f.P = o;   o += 16 * NC;
    f.AUX = o; o += kChainAuxBytes;
    // The replay's streams, all doubles (float terms are widened when written, one instruction
    // for all lanes, instead of inside the serial walk): lanes 0..4, 6, 7 read PX, PY, CPHF,
    // RMXF, LCL, LPW, LANG with one instruction, each stream starting on its own banks.
    unsigned dslots = 0u;
    f.PX = bank_place_c(o, dslots);   o = f.PX + 8 * NC;
    f.PY = bank_place_c(o, dslots);   o = f.PY + 8 * NC;
    f.CPHF = bank_place_c(o, dslots); o = f.CPHF + 8 * NC;
    f.RMXF = bank_place_c(o, dslots); o = f.RMXF + 8 * NC;
    f.LCL = bank_place_c(o, dslots);  o = f.LCL + 16 * L;
    // the Box-Muller pairs of the chain's 64-word Philox window (WaveRngLds, one chain per wave)
    f.RNG = o; o += L == 64 ? 512 : 0;
    f.end = o;
    return f;
}

inline MH_HD constexpr int fixed_cla(const FixedLds& f) { return (f.end + 15) & ~15; }

// with_off: the layout of the passes that evaluate OffLimitsCosts (final / evaluation). The
// instance-fixed part comes from fixed_lds(); the PairWise / Angle lists, clearance boxes and
// off-limits boxes (sized by R, C, N) follow at run-time offsets.
inline MH_HD ChainLds make_lds_layout(int n, int c, int r, int L, bool with_off = false) {
    const int NPL = npl_instance((n + L - 1) / L);
    const FixedLds f = fixed_lds(L, NPL);
    ChainLds l;
    l.h_room = f.h_room;
    l.h_obj = f.h_obj;
    l.h_frz = f.h_frz;
    l.h_clr = f.h_clr;
    int h = f.h_clr + round16((int)sizeof(RectShape) * (c > 0 ? c : 1));
    l.h_rel = h;  h += round16((int)sizeof(RelConst) * (r > 0 ? r : 1));
    l.h_rix = h;  h += round16(8 * (r > 0 ? r : 1));
    l.h_re = h;   h += 32 * (r > 0 ? r : 1);
    l.hdr = h;
    l.P = f.P;
    l.AUX = f.AUX;
    l.PX = f.PX;
    l.PY = f.PY;
    l.CPHF = f.CPHF;
    l.RMXF = f.RMXF;
    l.LCL = f.LCL;
    l.lst_r = ((r < 1 ? 1 : (r < L ? r : L)) + 3) & ~3;
    l.N4 = (n + 3) & ~3;
    int o = f.end;
    unsigned dslots = 0u;  // LPW / LANG on banks apart from the other replay streams
    dslots |= 1u << ((f.PX >> 4) & 15);
    dslots |= 1u << ((f.PY >> 4) & 15);
    dslots |= 1u << ((f.CPHF >> 4) & 15);
    dslots |= 1u << ((f.RMXF >> 4) & 15);
    dslots |= 1u << ((f.LCL >> 4) & 15);
    // the per-step Clearance arrays first: CLA at a compile-time offset (fixed_cla), NZ and PRE
    // from it and C, so the step kernel holds no scalar registers for them (config 3 111.0 ->
    // 110.1 ms per launch, the same trajectories)
    l.CLA = fixed_cla(f);            o = l.CLA + 16 * (c > 0 ? c : 1);
    l.NZ = o;                        o += 16 * (c > 0 ? c : 1);
    l.PRE = o;                       o += round16(4 * (c > 0 ? c : 1));
    l.LPW = bank_place(o, &dslots);  o = l.LPW + 8 * l.lst_r;
    l.LANG = bank_place(o, &dslots); o = l.LANG + 8 * l.lst_r;
    l.OFF = -1;
    if (with_off) {
        l.OFF = o;
        o += round16(16 * n);
    }
    o = round16(o);
    if ((o & 255) == 0) o += 16;  // spread the chains of one wave over the LDS banks
    l.stride = o;
    return l;
}

}  // namespace mh
