// mh_abi.cpp -- the C ABI of libmhgpu.so: KernelWrapper (Kernel.cu:873-984) and friends.
//
// Host side of the drop-in boundary. It validates the wire structs (the reference validates
// nothing and exits the host process on a CUDA error, helper_cuda.h:985-994), reduces the room
// to per-object device constants, owns device memory per session, and shards a KernelWrapper
// call over $MH_DEVICES (one host thread and one stream per device; chain c always draws from
// Philox subsequence c, so results do not depend on the device count).

#include <hip/hip_runtime.h>

#include <float.h>
#include <stddef.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <sys/mman.h>

#include <algorithm>
#include <future>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mh_launch.h"
#include "mh_math.h"

static_assert((int)mh::RNG_PHILOX == MH_RNG_PHILOX &&
                  (int)mh::RNG_CURAND_XORWOW == MH_RNG_CURAND_XORWOW, "RNG kinds");
static_assert((int)mh::TRACK_OFF == MH_TRACK_OFF && (int)mh::TRACK_LOWEST == MH_TRACK_LOWEST &&
                  (int)mh::TRACK_HIGHEST == MH_TRACK_HIGHEST,
              "device and ABI best-tracking modes");

namespace {

thread_local std::string g_last_error;
// The step kernel of this thread's last KernelWrapper call (mh_debug_wrapper_step): lanes per
// chain and kind as mh_session_geometry reports them; -1 before any call.
thread_local int g_wrapper_lanes = -1, g_wrapper_kind = -1;

void set_error(const std::string& e) { g_last_error = e; }

#define MH_TRY_HIP(expr)                                                                   \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess) {                                                            \
            set_error(std::string(#expr) + ": " + hipGetErrorString(_e));                  \
            return false;                                                                  \
        }                                                                                  \
    } while (0)

// Largest chunk of MH steps per launch: keeps one launch well under a second at N=64.
constexpr int kStepsPerLaunch = 1000;

struct Room {
    mh::DevRoom rm{};
    std::vector<mh::ObjConst> obj;
    std::vector<mh::ClrConst> clr;
    std::vector<mh::RelConst> rel;
    std::vector<float4> rele;  // [2][R] (mh::rel_est_consts)
    std::vector<double> cfg0;  // [6][N]
};

mh::RectShape make_shape(const vertex* v) {
    mh::RectShape s{};
    s.v0x = (float)v[0].x;
    s.xmin1 = std::min(v[1].x, std::min(v[2].x, v[3].x));
    s.xmax = std::max(std::max(v[0].x, v[1].x), std::max(v[2].x, v[3].x));
    s.ymin = std::min(std::min(v[0].y, v[1].y), std::min(v[2].y, v[3].y));
    s.ymax = std::max(std::max(v[0].y, v[1].y), std::max(v[2].y, v[3].y));
    return s;
}

bool validate(const relationshipStruct* rss, const relationshipAngleStruct* rsa,
              const positionAndRotation* cfg, const rectangle* clearances,
              const rectangle* offlimits, const vertex* vertices, const vertex* srect,
              const Surface* srf) {
    if (!srf) { set_error("srf is NULL"); return false; }
    const int n = srf->nObjs, c = srf->nClearances, nr = srf->nRelationships;
    char buf[160];
    if (n < 1) { snprintf(buf, sizeof buf, "nObjs must be >= 1 (got %d)", n); set_error(buf); return false; }
    if (c < 0 || c > n) {
        snprintf(buf, sizeof buf, "nClearances must be in [0, nObjs] (got %d)", c);
        set_error(buf);
        return false;
    }
    if (nr < 0) { set_error("nRelationships must be >= 0"); return false; }
    if (!cfg || !offlimits || !vertices || !srect) { set_error("NULL input array"); return false; }
    if ((nr > 0 && (!rss || !rsa)) || (c > 0 && !clearances)) { set_error("NULL input array"); return false; }
    const long nv = 4L * (c + n);
    bool any_free = false;
    for (int i = 0; i < n; ++i) {
        const int p = offlimits[i].point1Index;
        if (p < 0 || p + 3 >= nv) {
            snprintf(buf, sizeof buf, "offlimits[%d].point1Index out of range", i);
            set_error(buf);
            return false;
        }
        if (!cfg[i].frozen) any_free = true;
    }
    if (!any_free) { set_error("every object is frozen (the reference never terminates)"); return false; }
    for (int i = 0; i < c; ++i) {
        const int p = clearances[i].point1Index, q = clearances[i].SourceIndex;
        if (p < 0 || p + 3 >= nv) {
            snprintf(buf, sizeof buf, "clearances[%d].point1Index out of range", i);
            set_error(buf);
            return false;
        }
        if (q < 0 || q >= n) {
            snprintf(buf, sizeof buf, "clearances[%d].SourceIndex out of range", i);
            set_error(buf);
            return false;
        }
    }
    for (int i = 0; i < nr; ++i) {
        if (rss[i].SourceIndex < 0 || rss[i].SourceIndex >= n || rss[i].TargetIndex < 0 ||
            rss[i].TargetIndex >= n || rsa[i].SourceIndex < 0 || rsa[i].SourceIndex >= n ||
            rsa[i].TargetIndex < 0 || rsa[i].TargetIndex >= n) {
            snprintf(buf, sizeof buf, "relationship %d index out of range", i);
            set_error(buf);
            return false;
        }
    }
    return true;
}

// Host reduction of the room (every value computed exactly as the reference computes it on
// each call; see mh_device.h for what each field replaces).
bool build_room(const relationshipStruct* rss, const relationshipAngleStruct* rsa,
                const positionAndRotation* cfg, const rectangle* clearances,
                const rectangle* offlimits, const vertex* vertices, const vertex* srect,
                const Surface* srf, Room& out) {
    if (!validate(rss, rsa, cfg, clearances, offlimits, vertices, srect, srf)) return false;
    const int n = srf->nObjs, c = srf->nClearances, nr = srf->nRelationships;
    mh::DevRoom& rm = out.rm;
    rm.n = n;
    rm.c = c;
    rm.r = nr;
    rm.w_pw = srf->WeightPairWise;
    rm.w_vb = srf->WeightVisualBalance;
    rm.w_fp = srf->WeightFocalPoint;
    rm.w_sym = srf->WeightSymmetry;
    rm.w_ol = srf->WeightOffLimits;
    rm.w_cl = srf->WeightClearance;
    rm.w_sa = srf->WeightSurfaceArea;
    rm.fxf = (float)srf->focalX;
    rm.fyf = (float)srf->focalY;
    rm.ux = (float)mh_cos(srf->focalRot);  // Kernel.cu:290 (mh_math.h, as the oracle)
    rm.uy = (float)mh_sin(srf->focalRot);  // Kernel.cu:291
    rm.cxf = (float)(srf->centroidX / 2);
    rm.cyf = (float)(srf->centroidY / 2);
    double along = srf->focalX * rm.ux;
    along = along + srf->focalY * rm.uy;
    rm.along_f = along;
    rm.two_focal_rot = 2 * srf->focalRot;

    // Room box: minValue/maxValue(surfaceRectangle, 0, 0, 0), Kernel.cu:448-449,585-586.
    double rminx = DBL_MAX, rminy = DBL_MAX, rmaxx = -DBL_MAX, rmaxy = -DBL_MAX;
    for (int k = 0; k < 4; ++k) {
        rminx = std::min(rminx, srect[k].x);
        rminy = std::min(rminy, srect[k].y);
        rmaxx = std::max(rmaxx, srect[k].x);
        rmaxy = std::max(rmaxy, srect[k].y);
    }
    rm.rmin_x = rminx;
    rm.rmin_y = rminy;
    rm.rmax_x = rmaxx;
    rm.rmax_y = rmaxy;
    const float width = (float)(rmaxx - rminx);
    const float height = (float)(rmaxy - rminy);
    rm.sx = width / 16;
    rm.sy = height / 16;
    // Complement rectangles, Kernel.cu:343-364, rounded to float as the overlap sees them.
    const double comp[4][4] = {{-DBL_MAX, -DBL_MAX, DBL_MAX, rminy},
                               {-DBL_MAX, rminy, rminx, rmaxy},
                               {-DBL_MAX, rmaxy, DBL_MAX, DBL_MAX},
                               {rmaxx, rminy, DBL_MAX, rmaxy}};
    for (int k = 0; k < 4; ++k)
        for (int q = 0; q < 4; ++q) rm.comp[k][q] = (float)comp[k][q];

    out.obj.resize(n);
    float denom = 0;
    for (int i = 0; i < n; ++i) {
        mh::ObjConst& o = out.obj[i];
        o.off = make_shape(vertices + offlimits[i].point1Index);
        o.area = (float)(cfg[i].length * cfg[i].width);
        o.frozen = cfg[i].frozen ? 1 : 0;
        denom = denom + o.area;  // Kernel.cu:202, same order
    }
    rm.denom = denom;
    rm.inv_denom = 1.0f / denom;
    out.clr.resize(c > 0 ? c : 1);
    for (int i = 0; i < c; ++i) {
        out.clr[i].shape = make_shape(vertices + clearances[i].point1Index);
        out.clr[i].src = clearances[i].SourceIndex;
    }
    out.rel.resize(nr > 0 ? nr : 1);
    for (int i = 0; i < nr; ++i) {
        mh::RelConst& r = out.rel[i];
        r.start = rss[i].TargetRange.targetRangeStart;
        r.end = rss[i].TargetRange.targetRangeEnd;
        r.s = rss[i].SourceIndex;
        r.t = rss[i].TargetIndex;
        r.amin = rsa[i].angleMin;
        r.amax = rsa[i].angleMax;
        r.as = rsa[i].SourceIndex;
        r.at = rsa[i].TargetIndex;
        // the two range normalisers, in the device's double arithmetic (no contraction)
        r.norm_w = (mh::kTwoPI - (r.amax + (mh::kTwoPI - r.amin))) / 2.0;
        r.norm_n = (mh::kTwoPI - (r.amax - r.amin)) / 2.0;
    }
    out.rele.assign(2 * out.rel.size(), make_float4(0.f, 0.f, 0.f, 0.f));
    for (size_t i = 0; i < out.rel.size(); ++i)
        mh::rel_est_consts(out.rel[i], out.rele[i], out.rele[out.rel.size() + i]);
    out.cfg0.resize((size_t)mh::F_COUNT * n);
    for (int i = 0; i < n; ++i) {
        out.cfg0[mh::F_X * n + i] = cfg[i].x;
        out.cfg0[mh::F_Y * n + i] = cfg[i].y;
        out.cfg0[mh::F_Z * n + i] = cfg[i].z;
        out.cfg0[mh::F_RX * n + i] = cfg[i].rotX;
        out.cfg0[mh::F_RY * n + i] = cfg[i].rotY;
        out.cfg0[mh::F_RZ * n + i] = cfg[i].rotZ;
    }
    return true;
}

struct Geometry {
    int L, npl, waves;   // full-evaluation kernel (init, final, evaluation; step when !delta)
    bool few;            // step with OP_STEP_FEW (no register cap: too few chains to use it)
    bool spec;           // step with the speculative kernel (mh_spec.hip)
    int spec_h;          // its halves: 2 (16-node tree, 4 wavefronts per chain) or 1 (8, 2)
    bool spec_bound;     // its instance deciding on the bound where certain (177 VGPRs: 4 chains per CU)
    mh::ChainLds lay;    // init / step
    int waves_ol;
    mh::ChainLds lay_ol; // final / evaluation (with the OffLimits boxes)
    bool delta;          // step with the incremental kernel (mh_delta.hip)
    int dL, dwaves;
    mh::DeltaLds dlay;
};

// Incremental step kernel geometry: one chain per wavefront; the workgroup size (chains per
// workgroup, up to 12, 8 above 128 objects) that keeps the most chains resident per CU, as the runtime's occupancy
// calculator counts them (registers, LDS, waves), rounded down to whole waves per SIMD above
// four; ties go to fewer waves per workgroup. The
// kernel is latency-bound, so resident chains are its throughput (measured at N = 256: 1 to 5
// chains per CU gave 6.6e6 to 3.3e7 chain-steps/s, the launch time unchanged). It is the
// default step above N = 128 (measured, chain-steps/s full vs incremental: N = 100 1.21e8 /
// 1.15e8, N = 128 8.8e7 / 8.8e7, N = 192 2.0e7 / 5.0e7, N = 256 8.9e6 / 3.1e7). $MH_DELTA=0/1
// forces the choice; $MH_DELTA_WAVES pins the workgroup size.
void choose_delta_geometry(int n, int c, int r, int max_lds, Geometry& g) {
    g.dlay = mh::make_delta_layout(n, c, r);
    const char* e = getenv("MH_DELTA");
    g.delta = e && *e ? atoi(e) != 0 : n > 128;
    int want_w = getenv("MH_DELTA_WAVES") ? atoi(getenv("MH_DELTA_WAVES")) : 0;
    if (want_w != 0 && (want_w < 1 || want_w > mh::delta_max_waves(n))) {
        // (a tuning knob: clamped to the kernel's launch bound, never a silent kernel change)
        const int w = want_w < 1 ? 1 : mh::delta_max_waves(n);
        fprintf(stderr, "mhgpu: MH_DELTA_WAVES=%d is outside 1..%d for %d objects; using %d\n",
                want_w, mh::delta_max_waves(n), n, w);
        want_w = w;
    }
    int best_chains = -1;
    g.dL = 64;
    g.dwaves = 0;
    for (int w = 1; w <= mh::delta_max_waves(n); ++w) {  // (the kernel's launch bound)
        if (want_w && w != want_w) continue;
        const size_t b = mh::delta_lds_bytes(g.dlay, w);
        if (b > (size_t)max_lds) continue;
        int chains = mh::delta_blocks_per_cu(n, w, b) * w;
        // Whole waves per SIMD: a workgroup of 9 puts three chains on one SIMD, whose VALU then
        // paces the other eight (N = 256: 9 chains 6.16e7 chain-steps/s, 8 chains 6.59e7).
        if (!want_w && chains > 4) chains &= ~3;
        if (chains > best_chains) {
            best_chains = chains;
            g.dwaves = w;
        }
    }
    if (g.dwaves == 0 || best_chains <= 0) g.delta = false;  // does not fit: full evaluation
}

// `plain`: the session runs the plain step family (no best-of-chain tracking, no tempering, the
// Philox stream); only that family has the few-chains instance (launch() sends the others to
// launch_step_best / launch_step_xw).
bool choose_geometry(int n, int c, int r, int device, int64_t n_chains, bool plain, Geometry& g) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1)
        cus = 256;
    // waves the full-evaluation step keeps resident: four per SIMD (LDS-bound at N = 64)
    g.L = mh::choose_lanes(n, n_chains, 16LL * cus);
    g.npl = mh::choose_npl(n, g.L);
    if (g.npl > mh::max_npl()) {
        set_error("nObjs too large (max " + std::to_string(64 * mh::max_npl()) + ")");
        return false;
    }
    g.lay = mh::make_lds_layout(n, c, r, g.L);
    int max_lds = 0;
    if (hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess)
        max_lds = 64 * 1024;
    // Four waves per workgroup (one per SIMD) while that keeps at least two workgroups per CU.
    // Measured at N = 64 (chain-steps/s by waves per workgroup): 2: 2.70e8, 3: 2.84e8,
    // 4: 2.96e8, 5: 2.83e8, 8: 2.84e8 -- the runtime's occupancy optimum (7, more resident
    // chains) measured 2.50e8. $MH_WAVES (1..8) pins it for experiments.
    g.waves = 4;
    while (g.waves > 1 && mh::lds_bytes(g.lay, g.L, g.waves) > 80 * 1024) g.waves >>= 1;
    if (const char* e = getenv("MH_WAVES")) {
        const int w = atoi(e);
        if (w >= 1 && w <= 8 && mh::lds_bytes(g.lay, g.L, w) <= (size_t)max_lds) g.waves = w;
    }
    // At most two chains per SIMD: the step kernel's register cap (five resident waves per SIMD)
    // buys nothing, and its spills lengthen every step (config 2: 1.92e8 chain-steps/s uncapped
    // against 1.77e8). $MH_STEP_FEW=0/1 forces the choice.
    g.few = plain && g.L == 64 && g.npl <= 1 && n_chains <= 8LL * cus;
    if (const char* e = getenv("MH_STEP_FEW"))
        if (*e) g.few = plain && g.L == 64 && g.npl <= 1 && atoi(e) != 0;
    // Rooms of at most 8 objects up to 64 chains per CU: the speculative kernel (two wavefronts
    // per chain, 7 chains resident per CU) evaluates a tree of 8 proposal histories at once and
    // commits the realised path. Measured against the full-evaluation kernels at N = 8
    // (chain-steps/s, profiles/r05/r05g_*, r05h_*, r05i_*): 1,792 chains 7.56e8 / 3.78e8, 8,192
    // 7.76e8 / 4.47e8, 16,384 8.27e8 / 7.18e8, 24,576 8.24e8 / 1.39e9, 65,536 8.52e8 / 1.64e9
    // (the full kernel fills the GPU there). $MH_SPEC=0/1 forces the choice.
    g.spec = plain && mh::spec_fits(n, c, r) && n_chains <= 64LL * cus;
    if (const char* e = getenv("MH_SPEC"))
        if (*e) g.spec = plain && mh::spec_fits(n, c, r) && atoi(e) != 0;
    // At most two chains per CU (at most two of a chain's four wavefronts per SIMD), the 16-node
    // tree: 4.1 steps per batch instead of 3.2 for a batch ~21% longer. More chains share the
    // SIMDs, and the longer batch costs more than the steps gain. Measured at N = 8, ms per
    // 1,000-step launch, 8-node (H = 1) / 16-node (H = 2) tree (profiles/r06/r06e_spec_halves_ab.txt):
    // 256 chains 1.67 / 1.55, 512 chains 1.83 / 1.78, 1,024 chains (config 2) 1.93 / 2.28.
    // $MH_SPEC_H=1/2 forces the halves.
    g.spec_h = n_chains <= 2LL * cus ? 2 : 1;
    if (const char* e = getenv("MH_SPEC_H"))
        if (*e) g.spec_h = atoi(e) >= 2 ? 2 : 1;
    // Decisions on the bound (mh_spec.hip): the instance that takes them holds ~175 VGPRs, two
    // wavefronts per SIMD (4 chains per CU at one half, 2 at two: the dispatcher then spreads a
    // CU's wavefronts evenly over its SIMDs), and its batches trade the exact jobs and sums for
    // fp32 estimates. Measured at N = 8 (ms per 1,000-step launch, bound / exact,
    // profiles/r06/r06v_*): 256 chains 1.40 / 1.56, 1,024 chains (config 2) 1.73 / 1.98, 2,048
    // chains 3.37-3.85 / 3.68 (two rounds of chains). So up to four chains per CU.
    // $MH_SPEC_BOUND=0/1 forces it.
    g.spec_bound = n_chains <= 4LL * cus;
    if (const char* e = getenv("MH_SPEC_BOUND"))
        if (*e) g.spec_bound = atoi(e) != 0;
    g.lay_ol = mh::make_lds_layout(n, c, r, g.L, true);
    g.waves_ol = 4;
    while (g.waves_ol > 1 && mh::lds_bytes(g.lay_ol, g.L, g.waves_ol) > 80 * 1024) g.waves_ol >>= 1;
    if (mh::lds_bytes(g.lay_ol, g.L, g.waves_ol) > (size_t)max_lds) {
        set_error("room does not fit in LDS");
        return false;
    }
    choose_delta_geometry(n, c, r, max_lds, g);
    return true;
}

// The options every entry point resolves to (mh_options with defaults applied).
mh_options default_options(uint64_t seed) {
    mh_options o{};
    o.seed = seed;
    o.track_best = MH_TRACK_OFF;
    o.rng = MH_RNG_PHILOX;
    o.n_temps = 1;
    o.swap_interval = 1;
    o.beta_min = mh::kBeta;
    return o;
}

bool check_options(const mh_options* o) {
    if (o->track_best < MH_TRACK_OFF || o->track_best > MH_TRACK_HIGHEST) {
        set_error("mh_options.track_best must be MH_TRACK_OFF, MH_TRACK_LOWEST or MH_TRACK_HIGHEST");
        return false;
    }
    if (o->rng < MH_RNG_PHILOX || o->rng > MH_RNG_CURAND_XORWOW) {
        set_error("mh_options.rng must be MH_RNG_PHILOX or MH_RNG_CURAND_XORWOW");
        return false;
    }
    if (o->n_temps < 0 || o->n_temps > 1024) {
        set_error("mh_options.n_temps must be in [0, 1024]");
        return false;
    }
    if (o->n_temps > 1 && (o->swap_interval < 1 || !(o->beta_min > 0.0) ||
                           !(o->beta_min <= mh::kBeta))) {
        set_error("parallel tempering needs swap_interval >= 1 and 0 < beta_min <= 2");
        return false;
    }
    for (int k = 0; k < 4; ++k)
        if (o->reserved[k] != 0) {
            set_error("mh_options.reserved must be zero");
            return false;
        }
    return true;
}

uint64_t seed_from_env() {
    const char* s = getenv("MH_SEED");
    if (s && *s) return strtoull(s, nullptr, 0);
    return (uint64_t)time(nullptr);  // Kernel.cu:943
}

}  // namespace

struct mh_session {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t last = nullptr;    // the stream the session's latest work was queued on
    hipEvent_t done = nullptr;     // recorded on `last` after that work
    Room room;
    Geometry geo{};
    int64_t n_chains = 0, chain_offset = 0;
    uint64_t seed = 0;
    int track = mh::TRACK_OFF;
    int rng = mh::RNG_PHILOX;
    unsigned int* d_xw = nullptr;  // [n_chains][6] XORWOW states (rng == RNG_CURAND_XORWOW)
    int n_temps = 1;               // parallel tempering replicas per group
    int swap_interval = 1;
    int64_t steps_done = 0;        // MH steps run so far (exchange rounds fall on multiples)
    std::vector<double> ladder;    // [n_temps] inverse temperatures, ladder[0] = BETA
    double* d_ladder = nullptr;
    int* d_perm = nullptr;         // [n_chains] rung -> group-local chain (per group)
    mh::ObjConst* d_obj = nullptr;
    mh::ClrConst* d_clr = nullptr;
    mh::RelConst* d_rel = nullptr;
    float4* d_rele = nullptr;
    double* d_cfg0 = nullptr;
    double* d_st = nullptr;
    double* d_best = nullptr;  // [n_chains][6][N] best-of-chain configurations (track on)
    mh::ChainMeta* d_meta = nullptr;
    point* d_pts = nullptr;
    resultCosts* d_costs = nullptr;
    mh_summary* d_summary = nullptr;
    // Download staging: two pinned chunks the library allocates (hipHostMalloc) and owns. A
    // download DMAs chunk k into one while the host copies chunk k - 1 out of the other into the
    // caller's buffer, which is never page-locked (hipHostRegister) -- see copy_out.
    unsigned char* h_stage = nullptr;
    size_t stage_chunk = 0;
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    // Element capacities of the buffers above: a pooled session (KernelWrapper's cache) keeps
    // its buffers across calls and grows one only when a call needs more.
    size_t cap_obj = 0, cap_clr = 0, cap_rel = 0, cap_rele = 0, cap_cfg0 = 0, cap_st = 0, cap_best = 0,
           cap_xw = 0, cap_ladder = 0, cap_perm = 0, cap_meta = 0, cap_pts = 0, cap_costs = 0,
           cap_summary = 0;
    // The geometry's inputs (choose_geometry runs only when they change)
    bool geo_valid = false;
    int geo_n = -1, geo_c = -1, geo_r = -1;
    int64_t geo_chains = -1;
    bool geo_plain = false;
    std::string geo_env;  // the tuning overrides choose_geometry read (geometry_env)

    static float bound_slack() {
        const char* e = getenv("MH_BOUND_SLACK");
        const float v = e ? (float)atof(e) : 1.0f;
        return v >= 1.0f ? v : 1.0f;  // (a narrower allowance would not be a bound)
    }

    mh::LaunchArgs args() const {
        mh::LaunchArgs a{};
        a.rm = room.rm;
        a.objc = d_obj;
        a.clrc = d_clr;
        a.relc = d_rel;
        a.rele = d_rele;
        a.cfg = d_cfg0;
        a.st = d_st;
        a.meta = d_meta;
        a.pts = d_pts;
        a.costs = d_costs;
        a.n_chains = n_chains;
        a.chain_offset = chain_offset;
        a.seed = seed;
        a.iterations = 0;
        a.track = track;
        a.best = d_best;
        a.rng = rng;
        a.xw = d_xw;
        a.n_temps = n_temps;
        a.ladder = d_ladder;
        a.bound_slack = bound_slack();
        a.spec_bound = geo.spec_bound ? 1 : 0;
        a.lay = geo.lay;
        a.dlay = geo.dlay;
        return a;
    }
};

namespace {

void free_session(mh_session* s) {
    if (!s) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->done) (void)hipEventSynchronize(s->done);  // work queued on a caller's stream
    (void)hipFree(s->d_obj);
    (void)hipFree(s->d_clr);
    (void)hipFree(s->d_rel);
    (void)hipFree(s->d_rele);
    (void)hipFree(s->d_cfg0);
    (void)hipFree(s->d_st);
    (void)hipFree(s->d_best);
    (void)hipFree(s->d_xw);
    (void)hipFree(s->d_ladder);
    (void)hipFree(s->d_perm);
    (void)hipFree(s->d_meta);
    (void)hipFree(s->d_pts);
    (void)hipFree(s->d_costs);
    (void)hipFree(s->d_summary);
    if (s->h_stage) (void)hipHostFree(s->h_stage);
    for (hipEvent_t e : s->stage_ev)
        if (e) (void)hipEventDestroy(e);
    if (s->done) (void)hipEventDestroy(s->done);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    (void)hipSetDevice(prev);
    delete s;
}

// A device buffer of at least `count` elements: the one held if it is large enough, else a new
// one (a pooled session's earlier work on it is complete: it was downloaded and synchronised
// before the session went back to the pool).
template <class T>
bool ensure(T** p, size_t& cap, size_t count) {
    if (count == 0) count = 1;
    if (*p && cap >= count) return true;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    cap = 0;
    MH_TRY_HIP(hipMalloc((void**)p, sizeof(T) * count));
    cap = count;
    return true;
}

template <class T>
bool upload(T** dst, size_t& cap, const std::vector<T>& src, hipStream_t st) {
    if (!ensure(dst, cap, src.size())) return false;
    MH_TRY_HIP(hipMemcpyAsync(*dst, src.data(), sizeof(T) * src.size(), hipMemcpyHostToDevice, st));
    return true;
}

// Orders work about to be queued on `st` after everything the session queued before, on
// whichever stream that was (its own stream for the setup, a caller's stream for a run; the
// event was recorded there, so that stream may since have been destroyed -- and a new stream
// can reuse a destroyed one's handle, so the wait is made even when the handles are equal).
bool order_after_last(mh_session* s, hipStream_t st) {
    MH_TRY_HIP(hipStreamWaitEvent(st, s->done, 0));
    return true;
}

// Marks the end of the work just queued on `st`.
bool record_done(mh_session* s, hipStream_t st) {
    MH_TRY_HIP(hipEventRecord(s->done, st));
    s->last = st;
    return true;
}

// The environment overrides choose_geometry (and choose_lanes, choose_delta_geometry) reads. A
// pooled session keeps its geometry only while these are unchanged too, so a KernelWrapper call
// made after one of them changed runs the kernel it names, not the previous call's.
std::string geometry_env() {
    static const char* const kVars[] = {"MH_LANES", "MH_WAVES", "MH_STEP_FEW", "MH_SPEC",
                                        "MH_SPEC_H", "MH_SPEC_BOUND", "MH_DELTA",
                                        "MH_DELTA_WAVES"};
    std::string key;
    for (const char* v : kVars) {
        const char* e = getenv(v);
        key += e ? e : "-";
        key += '\x1f';
    }
    return key;
}

// Sets a session up for its room, chains and options. A pooled session (KernelWrapper's cache)
// comes here again for every call: its stream and event are kept, its buffers grow only when
// too small, and the geometry is chosen again only for another room shape or chain count.
bool session_init(mh_session* s) {
    MH_TRY_HIP(hipSetDevice(s->device));
    if (!s->stream) MH_TRY_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    if (!s->done) MH_TRY_HIP(hipEventCreateWithFlags(&s->done, hipEventDisableTiming));
    s->last = s->stream;
    s->steps_done = 0;
    const bool plain = s->track == mh::TRACK_OFF && s->n_temps <= 1 && s->rng == mh::RNG_PHILOX;
    const int rn = s->room.rm.n, rc = s->room.rm.c, rr = s->room.rm.r;
    const std::string env = geometry_env();
    if (!(s->geo_valid && s->geo_n == rn && s->geo_c == rc && s->geo_r == rr &&
          s->geo_chains == s->n_chains && s->geo_plain == plain && s->geo_env == env)) {
        s->geo_valid = false;
        if (!choose_geometry(rn, rc, rr, s->device, s->n_chains, plain, s->geo)) return false;
        s->geo_valid = true;
        s->geo_n = rn;
        s->geo_c = rc;
        s->geo_r = rr;
        s->geo_chains = s->n_chains;
        s->geo_plain = plain;
        s->geo_env = env;
    }
    if (!upload(&s->d_obj, s->cap_obj, s->room.obj, s->stream)) return false;
    if (!upload(&s->d_clr, s->cap_clr, s->room.clr, s->stream)) return false;
    if (!upload(&s->d_rel, s->cap_rel, s->room.rel, s->stream)) return false;
    if (!upload(&s->d_rele, s->cap_rele, s->room.rele, s->stream)) return false;
    if (!upload(&s->d_cfg0, s->cap_cfg0, s->room.cfg0, s->stream)) return false;
    const int64_t nc = s->n_chains > 0 ? s->n_chains : 1;
    const size_t n = (size_t)s->room.rm.n;
    if (!ensure(&s->d_st, s->cap_st, (size_t)mh::F_COUNT * n * nc)) return false;
    if (s->track != mh::TRACK_OFF && !ensure(&s->d_best, s->cap_best, (size_t)mh::F_COUNT * n * nc))
        return false;
    if (s->n_temps > 1) {
        if (!upload(&s->d_ladder, s->cap_ladder, s->ladder, s->stream)) return false;
        std::vector<int> perm((size_t)nc);
        for (int64_t i = 0; i < (int64_t)perm.size(); ++i) perm[(size_t)i] = (int)(i % s->n_temps);
        if (!ensure(&s->d_perm, s->cap_perm, perm.size())) return false;
        MH_TRY_HIP(hipMemcpy(s->d_perm, perm.data(), sizeof(int) * perm.size(), hipMemcpyHostToDevice));
    }
    if (s->rng == mh::RNG_CURAND_XORWOW) {
        if (!ensure(&s->d_xw, s->cap_xw, (size_t)6 * nc)) return false;
        MH_TRY_HIP(mh::launch_xorwow_init(s->seed, s->chain_offset, s->n_chains, s->d_xw, s->stream));
    }
    if (!ensure(&s->d_meta, s->cap_meta, (size_t)nc)) return false;
    if (!ensure(&s->d_pts, s->cap_pts, n * nc)) return false;
    if (!ensure(&s->d_costs, s->cap_costs, (size_t)nc)) return false;
    if (!ensure(&s->d_summary, s->cap_summary, 1)) return false;
    MH_TRY_HIP(mh::launch(mh::OP_INIT, s->args(), s->geo.L, s->geo.npl, s->geo.waves, s->stream));
    return record_done(s, s->stream);
}

hipStream_t pick_stream(const mh_session* s, void* stream) {
    return stream ? (hipStream_t)stream : s->stream;
}

bool session_run(mh_session* s, int iterations, hipStream_t st) {
    MH_TRY_HIP(hipSetDevice(s->device));
    if (!order_after_last(s, st)) return false;
    mh::LaunchArgs a = s->args();
    for (int done = 0; done < iterations;) {
        int chunk = std::min(kStepsPerLaunch, iterations - done);
        if (s->n_temps > 1)  // stop at the next exchange round
            chunk = (int)std::min<int64_t>(chunk, s->swap_interval - s->steps_done % s->swap_interval);
        a.iterations = chunk;
        if (s->geo.spec) MH_TRY_HIP(mh::launch_spec(a, s->geo.spec_h, st));
        else if (s->geo.delta) MH_TRY_HIP(mh::launch_delta(a, s->geo.dwaves, st));
        else MH_TRY_HIP(mh::launch(s->geo.few ? mh::OP_STEP_FEW : mh::OP_STEP, a, s->geo.L,
                                   s->geo.npl, s->geo.waves, st));
        done += chunk;
        s->steps_done += chunk;
        if (s->n_temps > 1 && s->steps_done % s->swap_interval == 0)
            MH_TRY_HIP(mh::launch_exchange(a, s->d_perm, (int)(s->steps_done / s->swap_interval), st));
    }
    return record_done(s, st);
}

bool session_finalize(mh_session* s, hipStream_t st) {
    MH_TRY_HIP(hipSetDevice(s->device));
    if (!order_after_last(s, st)) return false;
    mh::LaunchArgs a = s->args();
    a.lay = s->geo.lay_ol;
    if (s->track != mh::TRACK_OFF) a.st = s->d_best;  // report each chain's best configuration
    MH_TRY_HIP(mh::launch(mh::OP_FINAL, a, s->geo.L, s->geo.npl, s->geo.waves_ol, st));
    return record_done(s, st);
}

// Bytes per download staging chunk (two are held per session: 16 MB of pinned host memory).
constexpr size_t kStageChunk = 8u << 20;
// Host threads that copy one staged chunk out (chunks of at least kParMin bytes).
constexpr int kCopyThreads = 4;
constexpr size_t kParMin = 1u << 20;

// memcpy split over kCopyThreads threads (this one included) for large chunks: one thread
// copies ~6-10 GB/s, the PCIe DMA that fills the next chunk meanwhile runs at ~50 GB/s.
void par_memcpy(void* dst, const void* src, size_t bytes) {
    if (bytes < kParMin) {
        memcpy(dst, src, bytes);
        return;
    }
    const size_t part = ((bytes / kCopyThreads) + 63) & ~(size_t)63;
    std::thread th[kCopyThreads - 1];
    int started = 0;
    for (int t = 1; t < kCopyThreads; ++t) {
        const size_t off = part * (size_t)t;
        if (off >= bytes) break;
        const size_t len = std::min(part, bytes - off);
        th[started++] = std::thread([=] {
            memcpy(static_cast<unsigned char*>(dst) + off,
                   static_cast<const unsigned char*>(src) + off, len);
        });
    }
    memcpy(dst, src, std::min(part, bytes));
    for (int t = 0; t < started; ++t) th[t].join();
}

// Maps every page of a fresh host buffer (the result block KernelWrapper mallocs) ahead of the
// download, so the first-touch faults run while the GPU samples instead of inside the copy.
// Transparent huge pages where the system allows them; MADV_POPULATE_WRITE (Linux 5.14) maps the
// range in one call, else one write per page. The contents are unspecified until the download.
void prefault(void* p, size_t bytes) {
    if (bytes == 0) return;
    const uintptr_t pg = 4096, b = (uintptr_t)p, e = b + bytes;
    const uintptr_t ab = (b + pg - 1) & ~(pg - 1), ae = e & ~(pg - 1);
    if (ae > ab) {
#ifdef MADV_HUGEPAGE
        (void)madvise((void*)ab, ae - ab, MADV_HUGEPAGE);
#endif
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
        if (madvise((void*)ab, ae - ab, MADV_POPULATE_WRITE) == 0) {
            static_cast<volatile unsigned char*>(p)[0] = 0;  // (the partial pages at the ends)
            static_cast<volatile unsigned char*>(p)[bytes - 1] = 0;
            return;
        }
    }
    volatile unsigned char* c = static_cast<volatile unsigned char*>(p);
    for (uintptr_t a = b; a < e; a = (a & ~(pg - 1)) + pg) c[a - b] = 0;  // one write per page
    c[bytes - 1] = 0;
}

// The session's pinned staging chunks, at least min(bytes, kStageChunk) each.
bool ensure_stage(mh_session* s, size_t bytes) {
    const size_t want = std::min(bytes, kStageChunk);
    if (!s->stage_ev[0]) MH_TRY_HIP(hipEventCreateWithFlags(&s->stage_ev[0], hipEventDisableTiming));
    if (!s->stage_ev[1]) MH_TRY_HIP(hipEventCreateWithFlags(&s->stage_ev[1], hipEventDisableTiming));
    if (s->h_stage && s->stage_chunk >= want) return true;
    if (s->h_stage) (void)hipHostFree(s->h_stage);
    s->h_stage = nullptr;
    s->stage_chunk = 0;
    const size_t chunk = (want + 4095) & ~(size_t)4095;
    MH_TRY_HIP(hipHostMalloc((void**)&s->h_stage, 2 * chunk, hipHostMallocDefault));
    s->stage_chunk = chunk;
    return true;
}

// Copies `bytes` from device memory into a caller's host buffer, ordered after the session's
// work (the reference's plain D2H copies, Kernel.cu:959-960). The caller's memory is only ever
// written by the host: the DMA lands in the session's own pinned chunks and the host copies each
// chunk out while the next one is in flight. (Round 5 page-locked the caller's buffer instead --
// hipHostRegister on whatever heap pages it shared with the caller's other objects -- and saw two
// "illegal memory access" reports at this point; DESIGN.md section 7 "The round-5 download
// fault".) Thread-safe across sessions: each shard of a KernelWrapper call writes a disjoint
// slice through its own session's chunks.
bool copy_out(mh_session* s, void* host, const void* dev, size_t bytes) {
    if (bytes == 0) return true;
    hipStream_t st = s->stream;
    if (!order_after_last(s, st)) return false;
    // The session's kernels first, so that a failure is attributed to them and not to the copy.
    if (const hipError_t ek = hipStreamSynchronize(st); ek != hipSuccess) {
        set_error(std::string("the session's kernels failed before the download: ") +
                  hipGetErrorString(ek));
        return false;
    }
    if (!ensure_stage(s, bytes)) return false;
    const size_t chunk = s->stage_chunk;
    const size_t chunks = (bytes + chunk - 1) / chunk;
    auto len = [&](size_t k) { return std::min(chunk, bytes - k * chunk); };
    // Chunk k goes to staging half k & 1; that half's previous chunk (k - 2) was copied out by
    // the host in iteration k - 1, so it is free.
    for (size_t k = 0; k <= chunks; ++k) {
        if (k < chunks) {
            MH_TRY_HIP(hipMemcpyAsync(s->h_stage + (k & 1) * chunk,
                                      static_cast<const unsigned char*>(dev) + k * chunk, len(k),
                                      hipMemcpyDeviceToHost, st));
            MH_TRY_HIP(hipEventRecord(s->stage_ev[k & 1], st));
        }
        if (k > 0) {
            const size_t j = k - 1;
            MH_TRY_HIP(hipEventSynchronize(s->stage_ev[j & 1]));
            par_memcpy(static_cast<unsigned char*>(host) + j * chunk, s->h_stage + (j & 1) * chunk,
                       len(j));
        }
    }
    return record_done(s, st);
}

// The session's final points and costs, after all of its queued work (an event wait, so another
// session's work on the same device is not waited for).
bool session_download(mh_session* s, point* pts, resultCosts* costs) {
    MH_TRY_HIP(hipSetDevice(s->device));
    const size_t n = (size_t)s->room.rm.n;
    if (s->n_chains <= 0) return true;
    if (pts && !copy_out(s, pts, s->d_pts, sizeof(point) * n * s->n_chains)) return false;
    if (costs && !copy_out(s, costs, s->d_costs, sizeof(resultCosts) * s->n_chains)) return false;
    return true;
}

// ---- KernelWrapper's session cache -----------------------------------------------------------
// A KernelWrapper call runs one session per device: a stream and an event, a dozen device
// buffers, the geometry (occupancy queries), the room upload, then the launches and the copy
// back. Creating and destroying all of that on every call cost a fixed ~7 ms (round 4: config
// 2's shape took 12.6 ms per call for 5.3 ms of kernels). A call now borrows a session from a
// per-device pool and gives it back after its download: stream, event and buffers are reused
// (a buffer grows only when a call needs more) and the geometry is kept while the room's shape
// and the chain count stay the same. Thread-safe: a mutex per device, and concurrent calls
// borrow different sessions (at most kPoolKeep idle ones are kept per device). The pool is never
// destroyed implicitly: freeing device memory from a static destructor would run after the HIP
// runtime's own teardown, so the process's exit releases it, and a host application that shares
// the GPU calls KernelReleaseCache() to free the idle sessions earlier (a config-3-shaped call
// leaves ~0.3 GB per session on the device). $MH_WRAPPER_CACHE=0 turns the cache off.
constexpr int kPoolDevices = 64;
constexpr size_t kPoolKeep = 2;

struct SessionPool {
    std::mutex mu;
    std::vector<mh_session*> idle;
};

SessionPool* session_pools() {
    static SessionPool* pools = new SessionPool[kPoolDevices];
    return pools;
}

// (read on every call: turning the cache off later in a process takes effect at the next call)
bool wrapper_cache_on() {
    const char* e = getenv("MH_WRAPPER_CACHE");
    return !(e && *e && atoi(e) == 0);
}

// Frees every idle pooled session (their device buffers, streams and pinned staging); returns
// how many. Sessions borrowed by calls in flight go back to the pool as usual afterwards.
int release_pools() {
    int freed = 0;
    for (int d = 0; d < kPoolDevices; ++d) {
        SessionPool& p = session_pools()[d];
        std::vector<mh_session*> idle;
        {
            std::lock_guard<std::mutex> lk(p.mu);
            idle.swap(p.idle);
        }
        for (mh_session* s : idle) {
            free_session(s);
            ++freed;
        }
    }
    return freed;
}

bool configure_session(mh_session* s, const Room& room, int device, int64_t n_chains,
                       int64_t chain_offset, const mh_options& o);

// A set-up session for a KernelWrapper shard: an idle pooled one if the device has one.
mh_session* session_borrow(const Room& room, int device, int64_t n_chains, int64_t chain_offset,
                           const mh_options& o) {
    mh_session* s = nullptr;
    if (wrapper_cache_on() && device >= 0 && device < kPoolDevices) {
        SessionPool& p = session_pools()[device];
        std::lock_guard<std::mutex> lk(p.mu);
        if (!p.idle.empty()) {
            s = p.idle.back();
            p.idle.pop_back();
        }
    }
    if (!s) s = new mh_session();
    if (!configure_session(s, room, device, n_chains, chain_offset, o)) {
        std::string e = g_last_error;
        free_session(s);
        set_error(e);
        return nullptr;
    }
    return s;
}

// Back to the pool after a complete call (its work is downloaded and synchronised).
void session_give_back(mh_session* s) {
    if (!s) return;
    if (wrapper_cache_on() && s->device >= 0 && s->device < kPoolDevices) {
        SessionPool& p = session_pools()[s->device];
        std::lock_guard<std::mutex> lk(p.mu);
        if (p.idle.size() < kPoolKeep) {
            p.idle.push_back(s);
            return;
        }
    }
    free_session(s);
}

mh_session* session_create(const Room& room, int device, int64_t n_chains, int64_t chain_offset,
                           const mh_options& o) {
    mh_session* s = new mh_session();
    if (!configure_session(s, room, device, n_chains, chain_offset, o)) {
        std::string e = g_last_error;
        free_session(s);
        set_error(e);
        return nullptr;
    }
    return s;
}

// Options, room and chains into a session (new or pooled), then its set-up.
bool configure_session(mh_session* s, const Room& room, int device, int64_t n_chains,
                       int64_t chain_offset, const mh_options& o) {
    const int K = o.n_temps > 1 ? o.n_temps : 1;
    if (K > 1 && (n_chains % K != 0 || chain_offset % K != 0)) {
        set_error("parallel tempering: the chain count and offset must be multiples of n_temps");
        return false;
    }
    const uint64_t seed = o.seed;
    if (s->device != device) {  // (a pooled session stays on its device; a new one starts at 0)
        if (s->stream || s->done) {
            set_error("internal: a session cannot change device");
            return false;
        }
    }
    s->track = o.track_best;
    s->rng = o.rng;
    s->n_temps = K;
    s->swap_interval = o.swap_interval > 0 ? o.swap_interval : 1;
    s->ladder.resize((size_t)K);
    for (int k = 0; k < K; ++k)  // geometric from BETA (rung 0) down to beta_min
        s->ladder[(size_t)k] = k == 0 ? mh::kBeta
                                      : mh::kBeta * pow(o.beta_min / mh::kBeta, (double)k / (K - 1));
    s->device = device;
    s->room = room;
    s->n_chains = n_chains;
    s->chain_offset = chain_offset;
    s->seed = seed;
    return session_init(s);
}

// The devices a KernelWrapper call shards over: $MH_DEVICES ("all", or a comma list of device
// ids), else the current device. Unknown ids are an error, and so is a repeated id -- two shards
// on one device are not a multi-GPU run -- unless $MH_DEVICES_ALLOW_DUPLICATES=1 (the one-GPU
// test of the sharding path).
bool devices_from_env(int current, std::vector<int>& d) {
    d.clear();
    const char* s = getenv("MH_DEVICES");
    if (!s || !*s) {
        d.push_back(current);
        return true;
    }
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    if (strcmp(s, "all") == 0) {
        for (int i = 0; i < count; ++i) d.push_back(i);
    } else {
        const char* dup = getenv("MH_DEVICES_ALLOW_DUPLICATES");
        const bool allow_dup = dup && atoi(dup) != 0;
        std::string str(s);
        size_t pos = 0;
        while (pos <= str.size()) {
            size_t e = str.find(',', pos);
            if (e == std::string::npos) e = str.size();
            if (e > pos) {
                const std::string tok = str.substr(pos, e - pos);
                char* end = nullptr;
                const long v = strtol(tok.c_str(), &end, 10);
                if (!end || *end || v < 0 || v >= count) {
                    set_error("MH_DEVICES: '" + tok + "' is not a device id (this process sees " +
                              std::to_string(count) + " devices)");
                    return false;
                }
                if (!allow_dup && std::find(d.begin(), d.end(), (int)v) != d.end()) {
                    set_error("MH_DEVICES: device " + tok + " is listed twice");
                    return false;
                }
                d.push_back((int)v);
            }
            pos = e + 1;
        }
    }
    if (d.empty()) {
        set_error("MH_DEVICES names no device");
        return false;
    }
    return true;
}

// One device's share of a KernelWrapper call, run on its own host thread.
struct Shard {
    int device;
    int64_t begin, count;
    int lanes = -1, kind = -1;  // the step kernel its session ran (mh_session_geometry's codes)
    bool ok = false;
    std::string err;
};

result* wrapper_impl(relationshipStruct* rss, relationshipAngleStruct* rsa, positionAndRotation* cfg,
                     rectangle* clearances, rectangle* offlimits, vertex* vertices,
                     vertex* surfaceRectangle, Surface* srf, gpuConfig* gpuCfg,
                     const mh_options& opts) {
    if (!gpuCfg) { set_error("gpuCfg is NULL"); return nullptr; }
    if (gpuCfg->gridxDim < 1) { set_error("gpuConfig.gridxDim must be >= 1"); return nullptr; }
    if (gpuCfg->iterations < 0) { set_error("gpuConfig.iterations must be >= 0"); return nullptr; }
    Room room;
    if (!build_room(rss, rsa, cfg, clearances, offlimits, vertices, surfaceRectangle, srf, room))
        return nullptr;
    int current = 0;
    if (hipGetDevice(&current) != hipSuccess) {
        set_error("no HIP device available");
        return nullptr;
    }
    const int64_t chains = gpuCfg->gridxDim;
    const int iterations = gpuCfg->iterations;
    const size_t n = (size_t)srf->nObjs;
    std::vector<int> devs;
    if (!devices_from_env(current, devs)) return nullptr;
    if ((int64_t)devs.size() > chains) devs.resize((size_t)chains);

    point* pts = (point*)malloc(sizeof(point) * n * (size_t)chains);
    result* res = (result*)malloc(sizeof(result) * (size_t)chains);
    std::vector<resultCosts> costs((size_t)chains);
    if (!pts || !res) {
        free(pts);
        free(res);
        set_error("host allocation failed");
        return nullptr;
    }
    // Shard whole tempering groups (K = 1 without tempering).
    const int64_t K = opts.n_temps > 1 ? opts.n_temps : 1;
    if (chains % K != 0) {
        free(pts);
        free(res);
        set_error("parallel tempering: gridxDim must be a multiple of n_temps");
        return nullptr;
    }
    const int64_t groups = chains / K;
    if ((int64_t)devs.size() > groups) devs.resize((size_t)groups);
    std::vector<Shard> shards(devs.size());
    for (size_t k = 0; k < devs.size(); ++k) {
        shards[k].device = devs[k];
        shards[k].begin = K * (groups * (int64_t)k / (int64_t)devs.size());
        shards[k].count = K * (groups * (int64_t)(k + 1) / (int64_t)devs.size()) - shards[k].begin;
    }
    // The result block's pages are mapped on a host thread of their own while the shards'
    // kernels run; a shard downloads only after that (the mapping writes the pages).
    std::shared_future<void> mapped =
        std::async(std::launch::async, [=] { prefault(pts, sizeof(point) * n * (size_t)chains); })
            .share();
    auto work = [&](Shard& sh) {
        mh_session* s = session_borrow(room, sh.device, sh.count, sh.begin, opts);
        if (!s) {
            sh.err = g_last_error;
            mapped.wait();
            return;
        }
        (void)mh_session_geometry(s, &sh.lanes, nullptr, &sh.kind);
        sh.ok = session_run(s, iterations, s->stream) && session_finalize(s, s->stream);
        mapped.wait();
        sh.ok = sh.ok && session_download(s, pts + n * sh.begin, costs.data() + sh.begin);
        if (!sh.ok) {
            sh.err = g_last_error;
            free_session(s);  // (a failed session is not reused)
        } else {
            session_give_back(s);
        }
    };
    if (shards.size() == 1) {
        work(shards[0]);
        g_wrapper_lanes = shards[0].lanes;
        g_wrapper_kind = shards[0].kind;
    } else {
        std::vector<std::thread> th;
        for (auto& sh : shards) th.emplace_back(work, std::ref(sh));
        for (auto& t : th) t.join();
        g_wrapper_lanes = shards[0].lanes;
        g_wrapper_kind = shards[0].kind;
    }
    (void)hipSetDevice(current);
    for (auto& sh : shards) {
        if (!sh.ok) {
            free(pts);
            free(res);
            set_error("device " + std::to_string(sh.device) + ": " + sh.err);
            return nullptr;
        }
    }
    for (int64_t i = 0; i < chains; ++i) {
        res[i].points = pts + n * (size_t)i;
        res[i].costs = costs[(size_t)i];
    }
    g_last_error.clear();
    return res;
}

}  // namespace

extern "C" {

MH_API result* KernelWrapper(relationshipStruct* rss, relationshipAngleStruct* rsa,
                             positionAndRotation* cfg, rectangle* clearances, rectangle* offlimits,
                             vertex* vertices, vertex* surfaceRectangle, Surface* srf,
                             gpuConfig* gpuCfg) {
    return wrapper_impl(rss, rsa, cfg, clearances, offlimits, vertices, surfaceRectangle, srf,
                        gpuCfg, default_options(seed_from_env()));
}

MH_API result* KernelWrapperSeeded(relationshipStruct* rss, relationshipAngleStruct* rsa,
                                   positionAndRotation* cfg, rectangle* clearances,
                                   rectangle* offlimits, vertex* vertices, vertex* surfaceRectangle,
                                   Surface* srf, gpuConfig* gpuCfg, uint64_t seed) {
    return wrapper_impl(rss, rsa, cfg, clearances, offlimits, vertices, surfaceRectangle, srf,
                        gpuCfg, default_options(seed));
}

MH_API result* KernelWrapperEx(relationshipStruct* rss, relationshipAngleStruct* rsa,
                               positionAndRotation* cfg, rectangle* clearances,
                               rectangle* offlimits, vertex* vertices, vertex* surfaceRectangle,
                               Surface* srf, gpuConfig* gpuCfg, const mh_options* opts) {
    if (!opts)
        return wrapper_impl(rss, rsa, cfg, clearances, offlimits, vertices, surfaceRectangle,
                            srf, gpuCfg, default_options(seed_from_env()));
    if (!check_options(opts)) return nullptr;
    return wrapper_impl(rss, rsa, cfg, clearances, offlimits, vertices, surfaceRectangle, srf,
                        gpuCfg, *opts);
}

MH_API void KernelFreeResult(result* res) {
    if (!res) return;
    free(res[0].points);
    free(res);
}

MH_API const char* KernelLastError(void) { return g_last_error.c_str(); }

MH_API int mh_debug_wrapper_step(int* lanes_per_chain, int* kind) {
    if (lanes_per_chain) *lanes_per_chain = g_wrapper_lanes;
    if (kind) *kind = g_wrapper_kind;
    return g_wrapper_kind < 0 ? -1 : 0;
}

MH_API int KernelReleaseCache(void) {
    int current = 0;
    const bool have = hipGetDevice(&current) == hipSuccess;
    const int freed = release_pools();
    if (have) (void)hipSetDevice(current);
    return freed;
}

MH_API int KernelEvaluateCosts(const relationshipStruct* rss, const relationshipAngleStruct* rsa,
                               const positionAndRotation* cfgs, int n_cfgs,
                               const rectangle* clearances, const rectangle* offlimits,
                               const vertex* vertices, const vertex* surfaceRectangle,
                               const Surface* srf, resultCosts* out_costs) {
    if (n_cfgs < 0 || !out_costs || !cfgs) { set_error("bad arguments"); return -1; }
    Room room;
    if (!build_room(rss, rsa, cfgs, clearances, offlimits, vertices, surfaceRectangle, srf, room))
        return -1;
    if (n_cfgs == 0) return 0;
    const int n = srf->nObjs;
    std::vector<double> all((size_t)n_cfgs * mh::F_COUNT * n);
    for (int k = 0; k < n_cfgs; ++k) {
        const positionAndRotation* c = cfgs + (size_t)k * n;
        double* d = all.data() + (size_t)k * mh::F_COUNT * n;
        for (int i = 0; i < n; ++i) {
            d[mh::F_X * n + i] = c[i].x;
            d[mh::F_Y * n + i] = c[i].y;
            d[mh::F_Z * n + i] = c[i].z;
            d[mh::F_RX * n + i] = c[i].rotX;
            d[mh::F_RY * n + i] = c[i].rotY;
            d[mh::F_RZ * n + i] = c[i].rotZ;
        }
    }
    int device = 0;
    if (hipGetDevice(&device) != hipSuccess) { set_error("no HIP device available"); return -1; }
    mh_session* s = session_create(room, device, 0, 0, default_options(0));  // tables only
    if (!s) return -1;
    bool ok = true;
    double* d_cfgs = nullptr;
    resultCosts* d_out = nullptr;
    auto fail = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && ok) {
            set_error(std::string(what) + ": " + hipGetErrorString(e));
            ok = false;
        }
    };
    fail(hipMalloc((void**)&d_cfgs, sizeof(double) * all.size()), "hipMalloc");
    if (ok) fail(hipMalloc((void**)&d_out, sizeof(resultCosts) * n_cfgs), "hipMalloc");
    if (ok) fail(hipMemcpy(d_cfgs, all.data(), sizeof(double) * all.size(), hipMemcpyHostToDevice), "hipMemcpy");
    if (ok) {
        mh::LaunchArgs a = s->args();
        a.cfg = d_cfgs;
        a.costs = d_out;
        a.n_chains = n_cfgs;
        a.lay = s->geo.lay_ol;
        fail(mh::launch(mh::OP_EVAL, a, s->geo.L, s->geo.npl, s->geo.waves_ol, s->stream), "launch");
    }
    if (ok) fail(hipStreamSynchronize(s->stream), "hipStreamSynchronize");
    if (ok) fail(hipMemcpy(out_costs, d_out, sizeof(resultCosts) * n_cfgs, hipMemcpyDeviceToHost), "hipMemcpy");
    (void)hipFree(d_cfgs);
    (void)hipFree(d_out);
    free_session(s);
    return ok ? 0 : -1;
}

MH_API mh_session* mh_session_create(const relationshipStruct* rss,
                                     const relationshipAngleStruct* rsa,
                                     const positionAndRotation* cfg, const rectangle* clearances,
                                     const rectangle* offlimits, const vertex* vertices,
                                     const vertex* surfaceRectangle, const Surface* srf,
                                     int device, int64_t n_chains, int64_t chain_offset,
                                     uint64_t seed) {
    if (n_chains < 0 || chain_offset < 0) { set_error("negative chain count or offset"); return nullptr; }
    Room room;
    if (!build_room(rss, rsa, cfg, clearances, offlimits, vertices, surfaceRectangle, srf, room))
        return nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) {
        set_error("invalid HIP device " + std::to_string(device));
        return nullptr;
    }
    return session_create(room, device, n_chains, chain_offset, default_options(seed));
}

MH_API mh_session* mh_session_create_ex(const relationshipStruct* rss,
                                        const relationshipAngleStruct* rsa,
                                        const positionAndRotation* cfg,
                                        const rectangle* clearances, const rectangle* offlimits,
                                        const vertex* vertices, const vertex* surfaceRectangle,
                                        const Surface* srf, int device, int64_t n_chains,
                                        int64_t chain_offset, const mh_options* opts) {
    if (!opts) { set_error("opts is NULL"); return nullptr; }
    if (!check_options(opts)) return nullptr;
    if (n_chains < 0 || chain_offset < 0) { set_error("negative chain count or offset"); return nullptr; }
    Room room;
    if (!build_room(rss, rsa, cfg, clearances, offlimits, vertices, surfaceRectangle, srf, room))
        return nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) {
        set_error("invalid HIP device " + std::to_string(device));
        return nullptr;
    }
    return session_create(room, device, n_chains, chain_offset, *opts);
}

MH_API int mh_session_run(mh_session* s, int iterations, void* stream) {
    if (!s || iterations < 0) { set_error("bad arguments"); return -1; }
    return session_run(s, iterations, pick_stream(s, stream)) ? 0 : -1;
}

MH_API int mh_session_finalize(mh_session* s, void* stream) {
    if (!s) { set_error("NULL session"); return -1; }
    return session_finalize(s, pick_stream(s, stream)) ? 0 : -1;
}

MH_API int mh_session_download(mh_session* s, point* out_points, resultCosts* out_costs) {
    if (!s) { set_error("NULL session"); return -1; }
    return session_download(s, out_points, out_costs) ? 0 : -1;
}

MH_API int mh_session_current_costs(mh_session* s, resultCosts* out) {
    if (!s || !out) { set_error("bad arguments"); return -1; }
    if (hipSetDevice(s->device) != hipSuccess) { set_error("hipSetDevice failed"); return -1; }
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess && s->n_chains > 0)
        e = hipMemcpy2D(out, sizeof(resultCosts), reinterpret_cast<const char*>(s->d_meta) + offsetof(mh::ChainMeta, costs),
                        sizeof(mh::ChainMeta), sizeof(resultCosts), (size_t)s->n_chains, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        set_error(std::string("current costs: ") + hipGetErrorString(e));
        return -1;
    }
    return 0;
}

MH_API int mh_session_summary(mh_session* s, mh_summary* out) {
    if (!s || !out) { set_error("bad arguments"); return -1; }
    if (hipSetDevice(s->device) != hipSuccess) { set_error("hipSetDevice failed"); return -1; }
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = mh::launch_summary(s->d_costs, s->d_meta, s->n_chains, s->chain_offset, s->d_summary, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (e == hipSuccess) e = hipMemcpy(out, s->d_summary, sizeof(mh_summary), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        set_error(std::string("summary: ") + hipGetErrorString(e));
        return -1;
    }
    return 0;
}

MH_API int mh_session_geometry(const mh_session* s, int* lanes_per_chain, int* chains_per_workgroup,
                               int* incremental) {
    if (!s) { set_error("NULL session"); return -1; }
    const int L = (s->geo.delta || s->geo.spec) ? 64 : s->geo.L;  // the step kernel's shape
    const int w = s->geo.spec ? mh::spec_waves() : s->geo.delta ? s->geo.dwaves : s->geo.waves;
    if (lanes_per_chain)
        *lanes_per_chain = s->geo.spec ? 64 * mh::spec_waves_per_chain(s->geo.spec_h) : L;
    if (chains_per_workgroup) *chains_per_workgroup = w * (64 / L);
    if (incremental) *incremental = s->geo.spec ? 3 : s->geo.delta ? 1 : (s->geo.few ? 2 : 0);
    return 0;
}

MH_API int mh_session_occupancy(const mh_session* s, int* chains_per_cu) {
    if (!s || !chains_per_cu) { set_error("NULL argument"); return -1; }
    const auto& g = s->geo;
    int blocks = 0;
    if (g.spec) {
        *chains_per_cu = mh::spec_blocks_per_cu(g.spec_h, g.spec_bound) * mh::spec_waves();
    } else if (g.delta) {
        blocks = mh::delta_blocks_per_cu(s->room.rm.n, g.dwaves,
                                         mh::delta_lds_bytes(s->geo.dlay, g.dwaves));
        *chains_per_cu = blocks * g.dwaves;
    } else {
        blocks = mh::step_blocks_per_cu(g.L, g.npl, g.waves,
                                        mh::lds_bytes(s->geo.lay, g.L, g.waves), g.few);
        *chains_per_cu = blocks * g.waves * (64 / g.L);
    }
    return 0;
}

MH_API void mh_session_destroy(mh_session* s) { free_session(s); }

// Diagnostic: the Philox words, uniforms and normals a chain with this (seed, subsequence)
// draws, exactly as the chain kernel draws them. Returns 0 on success.
MH_API int mh_debug_rng(uint64_t seed, uint64_t subsequence, int n, unsigned int* out_u32,
                        float* out_uniform, float* out_normal) {
    return mh_debug_rng_ex(MH_RNG_PHILOX, seed, subsequence, n, out_u32, out_uniform, out_normal);
}

MH_API int mh_debug_rng_ex(int rng, uint64_t seed, uint64_t subsequence, int n,
                           unsigned int* out_u32, float* out_uniform, float* out_normal) {
    if (n < 0 || !out_u32 || !out_uniform || !out_normal || rng < MH_RNG_PHILOX ||
        rng > MH_RNG_CURAND_XORWOW) {
        set_error("bad arguments");
        return -1;
    }
    if (n == 0) return 0;
    unsigned int* d_u = nullptr;
    float *d_f = nullptr, *d_n = nullptr;
    hipError_t e = hipMalloc((void**)&d_u, sizeof(unsigned int) * n);
    if (e == hipSuccess) e = hipMalloc((void**)&d_f, sizeof(float) * n);
    if (e == hipSuccess) e = hipMalloc((void**)&d_n, sizeof(float) * n);
    if (e == hipSuccess) e = mh::launch_rng(rng, seed, subsequence, n, d_u, d_f, d_n, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out_u32, d_u, sizeof(unsigned int) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_uniform, d_f, sizeof(float) * n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_normal, d_n, sizeof(float) * n, hipMemcpyDeviceToHost);
    (void)hipFree(d_u);
    (void)hipFree(d_f);
    (void)hipFree(d_n);
    if (e != hipSuccess) {
        set_error(std::string("mh_debug_rng: ") + hipGetErrorString(e));
        return -1;
    }
    return 0;
}

MH_API int mh_debug_math(int fn, uint64_t start, uint64_t count, double* out) {
    if (fn < 0 || fn >= MH_PROBE_COUNT || !out || count > (1ull << 28)) {
        set_error("bad arguments");
        return -1;
    }
    if (count == 0) return 0;
    const size_t bytes = sizeof(double) * (size_t)mh_probe_width(fn) * (size_t)count;
    double* d = nullptr;
    hipError_t e = hipMalloc((void**)&d, bytes);
    if (e == hipSuccess) e = mh::launch_math(fn, start, count, d, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, d, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) {
        set_error(std::string("mh_debug_math: ") + hipGetErrorString(e));
        return -1;
    }
    return 0;
}

MH_API int mh_debug_collectives(int L, const float* v, const int* iv, int* out) {
    if (!(L == 8 || L == 16 || L == 32 || L == 64) || !v || !iv || !out) {
        set_error("bad arguments");
        return -1;
    }
    float* d_v = nullptr;
    int *d_iv = nullptr, *d_out = nullptr;
    hipError_t e = hipMalloc((void**)&d_v, sizeof(float) * 64);
    if (e == hipSuccess) e = hipMalloc((void**)&d_iv, sizeof(int) * 64);
    if (e == hipSuccess) e = hipMalloc((void**)&d_out, sizeof(int) * 17 * 64);
    if (e == hipSuccess) e = hipMemcpy(d_v, v, sizeof(float) * 64, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_iv, iv, sizeof(int) * 64, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = mh::launch_collectives(L, d_v, d_iv, d_out, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, d_out, sizeof(int) * 17 * 64, hipMemcpyDeviceToHost);
    (void)hipFree(d_v);
    (void)hipFree(d_iv);
    (void)hipFree(d_out);
    if (e != hipSuccess) {
        set_error(std::string("mh_debug_collectives: ") + hipGetErrorString(e));
        return -1;
    }
    return 0;
}

}  // extern "C"
