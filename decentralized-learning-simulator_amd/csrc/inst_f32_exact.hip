// inst_f32_exact.hip — instantiation unit: the kernels and host dispatch of these
// element policies (dispatch.hpp); compiled in parallel with the others.
#include "dispatch.hpp"

DLSIM_REDUCE_ENTRIES(template, dlsim::F32Exact)
