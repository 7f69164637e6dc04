// Fast-stream (PhiloxGen) InvMgmt run kernels: invmgmt.hip compiled again with
// INVSIM_IM_FAST_TU, which instantiates only im_run_kernel<..., PhiloxGen>
// and defines im_run_launch_ph (the parity TU's kernels stay there).
#define INVSIM_IM_FAST_TU
#include "invmgmt.hip"
