/*
 * mh_kernel.h -- C ABI of the MI355X Metropolis-Hastings interior-layout sampler.
 *
 * Drop-in boundary for the reference DLL surface
 *   KernelFolder/Kernel/Kernel.cu:873  extern "C" __declspec(dllexport) result* KernelWrapper(...)
 * The eleven wire structs below are byte-identical to Kernel.cu:43-149 on x86-64 (sizes and
 * offsets are static_assert-ed at the bottom of this header and again in the library).
 *
 * Ownership: KernelWrapper returns a host-malloc'd result[gridxDim]; every result[i].points
 * points into ONE malloc'd point[gridxDim * nObjs] block (as Kernel.cu:928,970-981 does).
 * Free it with KernelFreeResult(). On any error NULL is returned and KernelLastError()
 * describes it (the reference calls exit() inside the host process, helper_cuda.h:985-994).
 */
#ifndef MH_KERNEL_H_
#define MH_KERNEL_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define MH_API __attribute__((visibility("default")))
#else
#define MH_API
#endif

/* ---- wire structs: Kernel.cu:43-149 ------------------------------------------------------ */

typedef struct vertex { /* Kernel.cu:43-48 */
    double x;
    double y;
    double z;
} vertex;

typedef struct rectangle { /* Kernel.cu:50-57; only point1Index (4 consecutive vertices) and
                              SourceIndex (clearances only) are read, Kernel.cu:366-401,414 */
    int point1Index;
    int point2Index;
    int point3Index;
    int point4Index;
    int SourceIndex;
} rectangle;

typedef struct positionAndRotation { /* Kernel.cu:59-72 */
    double x;
    double y;
    double z;
    double rotX;
    double rotY;
    double rotZ;
#ifdef __cplusplus
    bool frozen;
#else
    _Bool frozen;
#endif
    double length;
    double width;
} positionAndRotation;

typedef struct targetRangeStruct { /* Kernel.cu:74-77 */
    double targetRangeStart;
    double targetRangeEnd;
} targetRangeStruct;

typedef struct relationshipStruct { /* Kernel.cu:79-85 */
    targetRangeStruct TargetRange;
    int SourceIndex;
    int TargetIndex;
    double DegreesOfAtrraction; /* spelling as in the reference; unused by the cost model */
} relationshipStruct;

typedef struct relationshipAngleStruct { /* Kernel.cu:87-92 */
    double angleMin;
    double angleMax;
    int SourceIndex;
    int TargetIndex;
} relationshipAngleStruct;

typedef struct Surface { /* Kernel.cu:94-117 */
    int nObjs;
    int nRelationships;
    int nClearances;
    float WeightFocalPoint;
    float WeightPairWise;
    float WeightVisualBalance;
    float WeightSymmetry;
    float WeightOffLimits;
    float WeightClearance;
    float WeightSurfaceArea;
    double centroidX;
    double centroidY;
    double focalX;
    double focalY;
    double focalRot;
} Surface;

typedef struct gpuConfig { /* Kernel.cu:119-127 */
    int gridxDim;   /* number of chains (one result per chain) */
    int gridyDim;   /* unused, as in the reference (Kernel.cu:946-947) */
    int blockxDim;  /* accepted and ignored: lanes per chain are chosen by the library */
    int blockyDim;  /* unused */
    int blockzDim;  /* unused */
    int iterations; /* MH steps per chain */
} gpuConfig;

typedef struct point { /* Kernel.cu:129-132 */
    float x, y, z, rotX, rotY, rotZ;
} point;

typedef struct resultCosts { /* Kernel.cu:134-144 */
    float totalCosts;
    float PairWiseCosts;
    float VisualBalanceCosts;
    float FocalPointCosts;
    float SymmetryCosts;
    float ClearanceCosts;
    float OffLimitsCosts;
    float SurfaceAreaCosts;
} resultCosts;

typedef struct result { /* Kernel.cu:146-149 */
    point* points;
    resultCosts costs;
} result;

/* ---- the reference export ---------------------------------------------------------------- */

/* Replaces Kernel.cu:873-984. Same name, parameter order and types. Runs gpuCfg->gridxDim
 * independent chains of gpuCfg->iterations MH steps each on the current HIP device and returns
 * every chain's final current configuration. Seed: $MH_SEED if set, else time(NULL)
 * (Kernel.cu:943). result[i].costs holds the cost components of that final configuration
 * (the reference leaves them uninitialised, Kernel.cu:852-861). Blocking. */
MH_API result* KernelWrapper(relationshipStruct* rss, relationshipAngleStruct* rsa,
                             positionAndRotation* cfg, rectangle* clearances,
                             rectangle* offlimits, vertex* vertices, vertex* surfaceRectangle,
                             Surface* srf, gpuConfig* gpuCfg);

/* ---- additive exports -------------------------------------------------------------------- */

/* KernelWrapper with an explicit 64-bit seed (chain c draws from Philox4x32-10 key=seed,
 * subsequence=c). Identical seeds give identical results. */
MH_API result* KernelWrapperSeeded(relationshipStruct* rss, relationshipAngleStruct* rsa,
                                   positionAndRotation* cfg, rectangle* clearances,
                                   rectangle* offlimits, vertex* vertices,
                                   vertex* surfaceRectangle, Surface* srf, gpuConfig* gpuCfg,
                                   uint64_t seed);

/* Options of the extended entry points. */
typedef enum mh_track_best {
    MH_TRACK_OFF = 0,     /* output = each chain's final current state (Kernel.cu:834-850) */
    MH_TRACK_LOWEST = 1,  /* output = the lowest-totalCosts configuration a chain proposed,
                             the reference's commented-out cfgBest (Kernel.cu:779-782, 808-816,
                             840-860: `starCosts->totalCosts < bestCosts->totalCosts`) */
    MH_TRACK_HIGHEST = 2  /* the same with `>`: the direction Accept climbs (Kernel.cu:706-713) */
} mh_track_best;

typedef enum mh_rng_kind {
    MH_RNG_PHILOX = 0,        /* rocRAND Philox4x32-10, key = seed, chain c = subsequence c */
    MH_RNG_CURAND_XORWOW = 1  /* cuRAND's XORWOW as the reference seeds it: chain c runs
                                 curand_init((unsigned)(seed + c), c, 0) (Kernel.cu:151-159,943)
                                 and draws curand_uniform / curand_normal (Kernel.cu:569-710) */
} mh_rng_kind;

typedef struct mh_options {
    uint64_t seed;         /* RNG seed (see mh_rng_kind) */
    int32_t track_best;    /* mh_track_best. The initial configuration is the first best; every
                              proposal (accepted or not) is compared before the accept test; ties
                              keep the earlier one. */
    int32_t rng;           /* mh_rng_kind */
    int32_t n_temps;       /* parallel tempering: replicas per group (0 or 1 = off). Chains
                              [g*K, (g+1)*K) form group g; chain g*K+k starts at rung k, whose
                              inverse temperature is beta_k = 2 * (beta_min / 2)^(k / (K-1)):
                              rung 0 is the reference's BETA = 2 (Kernel.cu:706-713). The chain
                              count must be a multiple of K. */
    int32_t swap_interval; /* MH steps between replica-exchange rounds (>= 1 with tempering) */
    double beta_min;       /* inverse temperature of the hottest rung, 0 < beta_min <= 2 */
    int32_t reserved[4];   /* must be zero */
} mh_options;

/* KernelWrapper with options (NULL = KernelWrapper's defaults with seed $MH_SEED/time). With
 * track_best != MH_TRACK_OFF, result[i] holds chain i's best configuration and its eight cost
 * components (OffLimits included, as bestCosts would hold them). With parallel tempering,
 * result[g*K + k] holds the replica that ends at rung k of group g, so result[g*K] are the
 * BETA = 2 samples. Exchange round t (after steps t*swap_interval, t = 1, 2, ...) tries the
 * rung pairs (k, k+1) with k = (t-1) mod 2, 2 + (t-1) mod 2, ...; the pair swaps rungs when
 * u < min(1, (float)exp((beta_k - beta_k+1) * (E_k+1 - E_k))), E = current totalCosts, u the
 * Philox uniform of (key = seed, subsequence = 2^63 + g, offset = (t-1)*K + k). */
MH_API result* KernelWrapperEx(relationshipStruct* rss, relationshipAngleStruct* rsa,
                               positionAndRotation* cfg, rectangle* clearances,
                               rectangle* offlimits, vertex* vertices, vertex* surfaceRectangle,
                               Surface* srf, gpuConfig* gpuCfg, const mh_options* opts);

/* Frees a KernelWrapper result (the points block and the array). NULL is a no-op. */
MH_API void KernelFreeResult(result* res);

/* Frees the device memory, streams and pinned staging that KernelWrapper keeps between calls
 * (at most two idle sessions per device; $MH_WRAPPER_CACHE=0 keeps none). Returns the number of
 * sessions freed. Calls in flight are unaffected. (No reference counterpart: the reference
 * allocates and leaks per call, Kernel.cu:926-967.) */
MH_API int KernelReleaseCache(void);

/* Text of the last error on the calling thread ("" if none). */
MH_API const char* KernelLastError(void);

/* Evaluates the reference cost model (Kernel.cu:516-550, OffLimits included in its component,
 * excluded from totalCosts as at :547) for n_cfgs configurations of nObjs objects each, laid
 * out back to back in cfgs, on the current device. Returns 0 on success. */
MH_API int KernelEvaluateCosts(const relationshipStruct* rss, const relationshipAngleStruct* rsa,
                               const positionAndRotation* cfgs, int n_cfgs,
                               const rectangle* clearances, const rectangle* offlimits,
                               const vertex* vertices, const vertex* surfaceRectangle,
                               const Surface* srf, resultCosts* out_costs);

/* ---- session API: device-resident chains (bench, multi-GPU sharding, resumable runs) ----- */

typedef struct mh_session mh_session;

typedef struct mh_summary {
    double sum_total;      /* sum over this session's chains of final totalCosts */
    float best_total;      /* max totalCosts (MH maximises, Kernel.cu:706-713) */
    int32_t pad;
    int64_t best_chain;    /* GLOBAL chain id of the best chain (lowest id on ties) */
    int64_t n_chains;
    int64_t accepted;      /* accepted proposals over all chains and steps so far */
} mh_summary;

/* Uploads the room tables to `device` and initialises n_chains chains with global ids
 * [chain_offset, chain_offset + n_chains): state := cfg, Philox(seed, subsequence = id),
 * initial costs. Returns NULL on error. */
MH_API mh_session* mh_session_create(const relationshipStruct* rss,
                                     const relationshipAngleStruct* rsa,
                                     const positionAndRotation* cfg, const rectangle* clearances,
                                     const rectangle* offlimits, const vertex* vertices,
                                     const vertex* surfaceRectangle, const Surface* srf,
                                     int device, int64_t n_chains, int64_t chain_offset,
                                     uint64_t seed);

/* mh_session_create with options (opts->seed replaces `seed`). With track_best on, every chain
 * keeps its best configuration on the device, and mh_session_finalize / download / summary
 * report the best configurations instead of the current ones. */
MH_API mh_session* mh_session_create_ex(const relationshipStruct* rss,
                                        const relationshipAngleStruct* rsa,
                                        const positionAndRotation* cfg,
                                        const rectangle* clearances, const rectangle* offlimits,
                                        const vertex* vertices, const vertex* surfaceRectangle,
                                        const Surface* srf, int device, int64_t n_chains,
                                        int64_t chain_offset, const mh_options* opts);

/* Enqueues `iterations` MH steps for every chain on `stream` (a hipStream_t; NULL = the
 * session's own stream). Chains resume exactly: k runs of m steps == one run of k*m steps. */
MH_API int mh_session_run(mh_session* s, int iterations, void* stream);

/* Enqueues the final-state pass (OffLimits component, float points) on `stream`. */
MH_API int mh_session_finalize(mh_session* s, void* stream);

/* Synchronous copies of the finalised chains (either pointer may be NULL). */
MH_API int mh_session_download(mh_session* s, point* out_points, resultCosts* out_costs);

/* Synchronous copy of the costs each chain carries for its current state: the costs its last
 * accepted proposal was judged by (OffLimitsCosts is 0: the step path does not evaluate it,
 * Kernel.cu:548). Equal to a fresh evaluation of the state in every other field. */
MH_API int mh_session_current_costs(mh_session* s, resultCosts* out_costs);

/* Reduces the finalised chains on the device to one mh_summary (synchronous). */
MH_API int mh_session_summary(mh_session* s, mh_summary* out);

/* Shape of the session's step kernel: lanes per chain, chains per workgroup, and whether it is
 * the incremental-evaluation kernel (1), the full-evaluation kernel (0), the full-evaluation
 * kernel's instance for launches of few chains (2: no register cap), or the speculative kernel
 * (3: rooms of at most 8 objects with few chains; 8 consecutive proposals per wavefront). Any
 * pointer may be NULL. */
MH_API int mh_session_geometry(const mh_session* s, int* lanes_per_chain,
                               int* chains_per_workgroup, int* incremental);

/* Chains of this session's step kernel that one CU keeps resident, as the runtime's occupancy
 * calculator counts them (registers, LDS and the wave limit of its launch shape). */
MH_API int mh_session_occupancy(const mh_session* s, int* chains_per_cu);

MH_API void mh_session_destroy(mh_session* s);

/* ---- diagnostics -------------------------------------------------------------------------- */

/* The first n Philox words, uniforms (curand_uniform stand-in) and normals (curand_normal
 * stand-in) that chain `subsequence` draws under `seed`, computed on the current device by the
 * same device code the chains use (each stream restarted at draw 0). Returns 0 on success. */
/* The group collectives the kernels use (top-2 / max-with-index / exclusive scan / max / sum
 * over groups of L = 8, 16, 32 or 64 lanes), run on the current device for the 64 lane values
 * v (floats) and iv (ints); out receives 9 x 64 ints (layout in mh_chain.hip). Returns 0. */
MH_API int mh_debug_collectives(int L, const float* v, const int* iv, int* out);

/* The step kernel the calling thread's last KernelWrapper* call ran (its first shard): lanes per
 * chain and kind, coded as mh_session_geometry codes them. Returns -1 before any call. (The
 * pooled sessions keep their kernel choice only while the room shape, chain count, options and
 * the tuning overrides $MH_LANES / $MH_WAVES / $MH_STEP_FEW / $MH_SPEC / $MH_DELTA /
 * $MH_DELTA_WAVES are unchanged; this lets a test see that.) */
MH_API int mh_debug_wrapper_step(int* lanes_per_chain, int* kind);

MH_API int mh_debug_rng(uint64_t seed, uint64_t subsequence, int n, unsigned int* out_u32,
                        float* out_uniform, float* out_normal);

/* mh_debug_rng for either stream (mh_rng_kind). For MH_RNG_CURAND_XORWOW the stream is
 * curand_init(seed, subsequence, 0) as given (the chains add their id to the seed). */
MH_API int mh_debug_rng_ex(int rng, uint64_t seed, uint64_t subsequence, int n,
                           unsigned int* out_u32, float* out_uniform, float* out_normal);

/* The project's transcendentals (metropolis-hastings-gpgpu_amd/csrc/mh_math.h, shared with the
 * test oracle) evaluated on the current device by the device code the chains use: probe `fn`
 * (MH_PROBE_* in mh_math.h: the Box-Muller log and sincos, cosf, cuRAND's log and sincos, atan2,
 * atan2f and exp on the chains' argument streams) at argument indices start .. start + count - 1
 * (count <= 2^28); out receives count x width doubles (width 2 for the sincos probes). */
MH_API int mh_debug_math(int fn, uint64_t start, uint64_t count, double* out);

#ifdef __cplusplus
} /* extern "C" */
#endif

/* ---- layout checks (x86-64 values recorded in SURVEY.md 8(b)) ---------------------------- */
#ifdef __cplusplus
#define MH_STATIC_ASSERT static_assert
#else
#define MH_STATIC_ASSERT _Static_assert
#endif
MH_STATIC_ASSERT(sizeof(vertex) == 24, "vertex");
MH_STATIC_ASSERT(sizeof(rectangle) == 20, "rectangle");
MH_STATIC_ASSERT(sizeof(positionAndRotation) == 72, "positionAndRotation");
MH_STATIC_ASSERT(offsetof(positionAndRotation, rotZ) == 40, "rotZ");
MH_STATIC_ASSERT(offsetof(positionAndRotation, frozen) == 48, "frozen");
MH_STATIC_ASSERT(offsetof(positionAndRotation, length) == 56, "length");
MH_STATIC_ASSERT(offsetof(positionAndRotation, width) == 64, "width");
MH_STATIC_ASSERT(sizeof(targetRangeStruct) == 16, "targetRangeStruct");
MH_STATIC_ASSERT(sizeof(relationshipStruct) == 32, "relationshipStruct");
MH_STATIC_ASSERT(offsetof(relationshipStruct, SourceIndex) == 16, "rs.SourceIndex");
MH_STATIC_ASSERT(offsetof(relationshipStruct, TargetIndex) == 20, "rs.TargetIndex");
MH_STATIC_ASSERT(offsetof(relationshipStruct, DegreesOfAtrraction) == 24, "rs.Degrees");
MH_STATIC_ASSERT(sizeof(relationshipAngleStruct) == 24, "relationshipAngleStruct");
MH_STATIC_ASSERT(offsetof(relationshipAngleStruct, SourceIndex) == 16, "ra.SourceIndex");
MH_STATIC_ASSERT(sizeof(Surface) == 80, "Surface");
MH_STATIC_ASSERT(offsetof(Surface, WeightFocalPoint) == 12, "WeightFocalPoint");
MH_STATIC_ASSERT(offsetof(Surface, WeightSurfaceArea) == 36, "WeightSurfaceArea");
MH_STATIC_ASSERT(offsetof(Surface, centroidX) == 40, "centroidX");
MH_STATIC_ASSERT(offsetof(Surface, focalRot) == 72, "focalRot");
MH_STATIC_ASSERT(sizeof(gpuConfig) == 24, "gpuConfig");
MH_STATIC_ASSERT(sizeof(point) == 24, "point");
MH_STATIC_ASSERT(sizeof(resultCosts) == 32, "resultCosts");
MH_STATIC_ASSERT(sizeof(result) == 40, "result");
MH_STATIC_ASSERT(offsetof(result, costs) == 8, "result.costs");
MH_STATIC_ASSERT(sizeof(mh_summary) == 40, "mh_summary");
MH_STATIC_ASSERT(sizeof(mh_options) == 48, "mh_options");
MH_STATIC_ASSERT(offsetof(mh_options, beta_min) == 24, "mh_options.beta_min");

#endif /* MH_KERNEL_H_ */
