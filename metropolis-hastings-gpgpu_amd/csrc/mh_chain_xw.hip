// mh_chain_xw.hip -- the full-evaluation step kernels of mh_chain.hip drawing from the cuRAND
// XORWOW stream (mh_options.rng = MH_RNG_CURAND_XORWOW), best-of-chain tracking compiled in.
// A separate translation unit so the step-kernel families compile in parallel.
#define MH_CHAIN_STEP_TU OP_STEP_XW
#define MH_CHAIN_STEP_LAUNCH launch_step_xw
#include "mh_chain.hip"
