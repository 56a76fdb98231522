// mh_launch.h -- launch interface between the host library (mh_abi.cpp) and the HIP kernels
// (mh_chain.hip: full evaluation; mh_delta.hip: incremental step).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "mh_device.h"
#include "../../include/mh_kernel.h"

namespace mh {

// OP_STEP_FEW: OP_STEP compiled without the step kernel's register cap, for launches with too few
// chains to use the resident waves the cap buys (mh_abi.cpp choose_geometry; one chain per
// wavefront, one object per lane only).
enum Op { OP_INIT = 0, OP_STEP = 1, OP_FINAL = 2, OP_EVAL = 3, OP_STEP_XW = 4, OP_STEP_T = 5,
          OP_STEP_FEW = 6 };

// Which stream the chains draw from (mh_options.rng).
enum RngKind { RNG_PHILOX = 0, RNG_CURAND_XORWOW = 1 };

struct LaunchArgs {
    DevRoom rm;
    const ObjConst* objc;
    const ClrConst* clrc;
    const RelConst* relc;
    const float4* rele;      // [2][R] the relationships' fp32 estimate constants (rel_est_consts)
    const double* cfg;       // OP_INIT: [6][N] initial pose; OP_EVAL: [n_chains][6][N]
    double* st;              // [n_chains][6][N] chain poses
    ChainMeta* meta;         // [n_chains]
    point* pts;              // OP_FINAL: [n_chains][N]
    resultCosts* costs;      // OP_FINAL / OP_EVAL: [n_chains]
    int64_t n_chains;
    int64_t chain_offset;    // global id of local chain 0 (Philox subsequence)
    uint64_t seed;
    int iterations;
    int track;               // TRACK_OFF / TRACK_LOWEST / TRACK_HIGHEST
    double* best;            // [n_chains][6][N] best-of-chain configurations (track != 0)
    int rng;                 // RngKind
    int n_temps;             // parallel tempering replicas per group (1 = off)
    const double* ladder;    // [n_temps] inverse temperatures (n_temps > 1)
    unsigned int* xw;        // [n_chains][6] XORWOW states {d, x0..x4} (rng == RNG_CURAND_XORWOW)
    int spec_bound;          // speculative kernel: decide on the bound where it is certain
                             // (1, default; $MH_SPEC_BOUND=0: every node's exact costs)
    float bound_slack;       // diagnostic: widens the step bound's error allowance ($MH_BOUND_SLACK,
                             // default 1; the tests use it to send many steps down the exact paths)
    ChainLds lay;
    DeltaLds dlay;           // incremental step kernel (mh_delta.hip)
};

int choose_lanes(int n, int64_t n_chains, int64_t resident_waves);
int choose_npl(int n, int L);
int max_npl();
size_t lds_bytes(const ChainLds& lay, int L, int waves_per_wg);
hipError_t launch(int op, const LaunchArgs& a, int L, int npl, int waves_per_wg, hipStream_t s);
size_t delta_lds_bytes(const DeltaLds& lay, int waves_per_wg);
hipError_t launch_delta(const LaunchArgs& a, int waves_per_wg, hipStream_t s);
int delta_blocks_per_cu(int n, int waves_per_wg, size_t lds_bytes);
int delta_max_waves(int n);  // chains per workgroup the incremental kernel admits
int step_blocks_per_cu(int L, int npl, int waves_per_wg, size_t lds_bytes, bool few);
hipError_t launch_summary(const resultCosts* costs, const ChainMeta* meta, int64_t n,
                          int64_t chain_offset, mh_summary* out, hipStream_t s);
hipError_t launch_collectives(int L, const float* v, const int* iv, int* out, hipStream_t s);
hipError_t launch_step_xw(const LaunchArgs& a, int L, int npl, int waves_per_wg, hipStream_t s);
hipError_t launch_step_best(const LaunchArgs& a, int L, int npl, int waves_per_wg, hipStream_t s);
hipError_t launch_rng(int kind, uint64_t seed, uint64_t subsequence, int n, unsigned int* u32,
                      float* uni, float* nrm, hipStream_t s);
hipError_t launch_exchange(const LaunchArgs& a, int* perm, int round, hipStream_t s);
hipError_t launch_math(int fn, uint64_t start, uint64_t count, double* out, hipStream_t s);
// The speculative step kernel (mh_spec.hip): rooms of at most 8 objects and 16 relationships;
// a chain's 2 * halves wavefronts evaluate a tree of 8 * halves proposal histories at once.
bool spec_fits(int n, int c, int r);
int spec_waves();                       // chains per workgroup of the speculative kernel
int spec_waves_per_chain(int halves);   // its wavefronts per chain
size_t spec_lds_bytes(int halves);
int spec_blocks_per_cu(int halves, bool bound);
hipError_t launch_spec(const LaunchArgs& a, int halves, hipStream_t s);
hipError_t launch_xorwow_init(uint64_t seed, int64_t chain_offset, int64_t n, unsigned int* xw,
                              hipStream_t s);

}  // namespace mh
