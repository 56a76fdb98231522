// mh_chain_xw.hip -- the full-evaluation step kernels of mh_chain.hip instantiated with the
// cuRAND XORWOW stream (mh_options.rng = MH_RNG_CURAND_XORWOW). A separate translation unit so
// the two sets of step kernels compile in parallel.
#define MH_CHAIN_XW_TU 1
#include "mh_chain.hip"
