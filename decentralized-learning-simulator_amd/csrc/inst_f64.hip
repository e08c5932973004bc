// inst_f64.hip — instantiation unit: the kernels and host dispatch of these
// element policies (dispatch.hpp); compiled in parallel with the others.
#include "dispatch.hpp"

DLSIM_F64_ENTRIES(template, dlsim::F64Exact)
DLSIM_F64_ENTRIES(template, dlsim::F64Fast)
DLSIM_CHUNK_ENTRIES(template, dlsim::F64Mean)
