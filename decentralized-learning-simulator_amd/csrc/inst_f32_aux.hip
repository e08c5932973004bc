// inst_f32_aux.hip — instantiation unit: the kernels and host dispatch of these
// element policies (dispatch.hpp); compiled in parallel with the others.
#include "dispatch.hpp"

DLSIM_REDUCE_ENTRIES(template, dlsim::F32Fast)
DLSIM_MEAN_ENTRIES(template, dlsim::F32Mean)
DLSIM_PROBE_ENTRIES(template, dlsim::XorProbe<4>)
