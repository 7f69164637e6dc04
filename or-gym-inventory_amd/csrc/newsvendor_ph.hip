// Fast-stream (PhiloxGen) Newsvendor kernels: newsvendor.hip compiled again
// with INVSIM_NV_FAST_TU, which instantiates the lookahead step, rollout and
// run kernels on PhiloxGen and defines nv_run_launch_ph (the parity TU's
// kernels stay there).
#define INVSIM_NV_FAST_TU
#include "newsvendor.hip"
