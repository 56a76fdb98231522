// mh_chain_best.hip -- the full-evaluation step kernels of mh_chain.hip with best-of-chain
// tracking compiled in (mh_options.track_best != MH_TRACK_OFF, Philox stream). The plain step
// kernels in mh_chain.hip carry no tracking code at all.
#define MH_CHAIN_STEP_TU OP_STEP_T
#define MH_CHAIN_STEP_LAUNCH launch_step_best
#include "mh_chain.hip"
