/*
 * mh_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's hot path (KernelFolder/Kernel/Kernel.cu:162-828) used as
 * the parity checker for the HIP sampler. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product (libmhgpu.so / KernelWrapper) never links
 * or calls it and fails loudly without its HIP kernels.
 *
 * Pinning: the reference itself is unbuildable in this image (Kernel.cu includes
 * <cuda_runtime.h> and <curand_kernel.h>, which the image lacks; stand-in headers are not
 * allowed), so this restatement is pinned on the known-answer test recorded in SURVEY.md 8(c)
 * (the reference's own Costs() on the main() fixture, Kernel.cu:1007-1166) plus hand-derived
 * analytic cases in tests/. The RNG boundary (cuRAND XORWOW, Kernel.cu:19,159) is replaced by
 * rocRAND's Philox4x32-10 stream, restated here and checked bit-for-bit against the device.
 */
#ifndef MH_ORACLE_H_
#define MH_ORACLE_H_

#include <stdint.h>
#include "../include/mh_kernel.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The eight KernelWrapper inputs that define a room (Kernel.cu:873). */
typedef struct orc_room {
    const relationshipStruct* rs;
    const relationshipAngleStruct* ra;
    const rectangle* clearances;
    const rectangle* offlimits;
    const vertex* vertices;
    const vertex* surfaceRectangle;
    const Surface* srf;
} orc_room;

/* rocRAND philox4x32_10_engine state (rocrand_philox4x32_10.h) plus the Box-Muller cache. */
typedef struct orc_rng {
    uint32_t counter[4];
    uint32_t result[4];
    uint32_t key[2];
    uint32_t substate;
    int32_t bm_has;
    float bm_val;
    int32_t kind;    /* 0 Philox; ORC_XORWOW_CURAND / ORC_XORWOW_ROCRAND: the xorwow below */
    uint32_t xw[6];  /* xorwow {d, x0..x4} */
} orc_rng;

/* XORWOW seeding constants: cuRAND's (the reference's generator, Kernel.cu:19,159) or
 * rocRAND's (rocrand_xorwow.h; used only to pin the recurrence and the subsequence jump against
 * rocRAND's own engine, tests/golden/xorwow_rocrand.cpp). */
#define ORC_XORWOW_CURAND 1
#define ORC_XORWOW_ROCRAND 2

/* 0 on success, negative on a validation error (message via orc_last_error). */
int orc_validate(const orc_room* room, const positionAndRotation* cfg);
const char* orc_last_error(void);

/* Costs() of Kernel.cu:516-550 on one configuration of srf->nObjs objects. */
void orc_costs(const orc_room* room, const positionAndRotation* cfg, resultCosts* out);

/* Individual terms (raw, unweighted), for term-level tests. */
double orc_visual_balance(const orc_room* room, const positionAndRotation* cfg);
double orc_pairwise(const orc_room* room, const positionAndRotation* cfg);
double orc_pairwise_angle(const orc_room* room, const positionAndRotation* cfg);
double orc_focal_point(const orc_room* room, const positionAndRotation* cfg);
float orc_symmetry(const orc_room* room, const positionAndRotation* cfg);
float orc_clearance(const orc_room* room, const positionAndRotation* cfg);
float orc_surface_area(const orc_room* room, const positionAndRotation* cfg);
float orc_off_limits(const orc_room* room, const positionAndRotation* cfg);

/* RNG stream (seed, subsequence) as the device sees it. */
void orc_rng_init(orc_rng* r, uint64_t seed, uint64_t subsequence);
uint32_t orc_rng_next(orc_rng* r);
float orc_rng_uniform(orc_rng* r);
float orc_rng_normal(orc_rng* r);
void orc_philox_stream(uint64_t seed, uint64_t subsequence, uint32_t* out, int n);
/* curand_init(seed, subsequence, 0) for a curandStateXORWOW (kind ORC_XORWOW_CURAND), or the
 * rocRAND engine's equivalent (ORC_XORWOW_ROCRAND). orc_rng_next / _uniform / _normal then draw
 * curand(), curand_uniform() and curand_normal(). */
void orc_rng_init_xorwow(orc_rng* r, uint64_t seed, uint64_t subsequence, int kind);
/* Philox stream (seed, subsequence) started at draw `offset` (rocrand_init's offset). */
void orc_rng_init_offset(orc_rng* r, uint64_t seed, uint64_t subsequence, uint64_t offset);
/* Random123 philox4x32 with 10 rounds on one (counter, key) block, for KAT vectors. */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* generateRandomIntInRange (Kernel.cu:566-574) and the object pick with its frozen redraw
 * (Kernel.cu:598-602; index nObjs counts as frozen). */
int orc_rand_int(orc_rng* r, int max, int min);
int orc_pick_object(const positionAndRotation* cfg, int n, orc_rng* r);
/* How many times pick_object drew index nObjs (u == 1.0f) in this process; reset if asked. */
long long orc_index_n_draws(int reset);
/* Accept draws of u == 1.0f against an uphill proposal seen in this process (diagnostic). */
long long orc_u1_uphill_draws(int reset);
/* OffLimits in every step's Costs() (1, default: the reference's loop) or only for the output
 * configurations (0: identical outputs, faster). Process-wide. */
void orc_set_step_offlimits(int on);

/* One proposal (Kernel.cu:576-704) applied in place to cfg (nObjs entries). */
void orc_propose(const orc_room* room, positionAndRotation* cfg, orc_rng* r);
/* Accept rule of Kernel.cu:706-713. */
int orc_accept(double cost_star, double cost_cur, orc_rng* r);
/* The same at inverse temperature beta (parallel tempering). */
int orc_accept_at(double cost_star, double cost_cur, double beta, orc_rng* r);

/* Runs chains [chain_begin, chain_begin + n_chains) of the defined single-proposer chain
 * (Kernel.cu:777-828) for `iterations` steps on `nthreads` host threads. out_points holds
 * n_chains * nObjs points, out_costs n_chains entries, out_accepted n_chains counts (any of the
 * three may be NULL). Returns 0 on success. */
int orc_run_chains(const orc_room* room, const positionAndRotation* cfg, uint64_t seed,
                   int64_t chain_begin, int64_t n_chains, int iterations, int nthreads,
                   point* out_points, resultCosts* out_costs, int64_t* out_accepted);

/* Same as orc_run_chains but returns the full final double-precision state per chain
 * (n_chains * nObjs entries) -- used to check device trajectories bit for bit. */
int orc_run_chains_state(const orc_room* room, const positionAndRotation* cfg, uint64_t seed,
                         int64_t chain_begin, int64_t n_chains, int iterations, int nthreads,
                         positionAndRotation* out_state, resultCosts* out_costs,
                         int64_t* out_accepted);

/* orc_run_chains_state with the options of KernelWrapperEx (include/mh_kernel.h): seed and
 * best-of-chain tracking. With tracking on, out_state / out_costs hold each chain's best
 * configuration and its costs. */
/* opts->rng == MH_RNG_CURAND_XORWOW: chain c draws from curand_init((uint32_t)(seed + c), c, 0)
 * as Kernel.cu:151-159,943 seeds thread c. opts->n_temps > 1: parallel tempering as
 * KernelWrapperEx defines it (include/mh_kernel.h); outputs are in rung order per group
 * (out_accepted stays in chain order). */
int orc_run_chains_ex(const orc_room* room, const positionAndRotation* cfg,
                      const mh_options* opts, int64_t chain_begin, int64_t n_chains,
                      int iterations, int nthreads, positionAndRotation* out_state,
                      resultCosts* out_costs, int64_t* out_accepted);

/* The numerics probes of mh_math.h (MH_PROBE_*): out receives count x width doubles, probe
 * `fn` at argument indices start .. start + count - 1, on `nthreads` threads -- the values the
 * device diagnostic mh_debug_math must reproduce bit for bit. */
int orc_math_eval(int fn, uint64_t start, uint64_t count, int nthreads, double* out);

/* The same probes evaluated with the C library's log / sin / cos / atan2 / exp instead of
 * mh_math.h (the oracle's math before round 4), to report how far the two libraries differ. */
int orc_math_eval_libm(int fn, uint64_t start, uint64_t count, int nthreads, double* out);

/* mh_math.h's functions on given arguments: which = 0 log, 1 exp, 2 sin, 3 cos, 4 atan2(a, b),
 * 5 sin through the medium-range reduction only (|a| <= 2^20 pi/2). */
int orc_math_apply(int which, const double* a, const double* b, int64_t n, double* out);

#ifdef __cplusplus
}
#endif
#endif /* MH_ORACLE_H_ */
