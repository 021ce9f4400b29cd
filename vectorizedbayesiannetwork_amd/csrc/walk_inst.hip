// walk_inst.hip — one kind-set instantiation of vbn_walk_kernel (vbn_walk_impl.h) and its
// launcher, compiled once per kind set with -DVBN_INST_KM=<set> (Makefile), so the sets build
// in parallel.  vbn_walk.hip's vbn_hip_walk picks the launcher.
#include "vbn_walk_impl.h"

#ifndef VBN_INST_KM
#error "compile with -DVBN_INST_KM=<kind set>"
#endif

extern "C" hipError_t VBN_LAUNCHER(VBN_INST_KM)(const vbn_walk_args* a, dim3 grid, dim3 block, size_t lds,
                                                hipStream_t st) {
  hipLaunchKernelGGL(vbn_walk_kernel<(unsigned)VBN_INST_KM>, grid, block, lds, st, *a, a->params, a->steps,
                     a->in_cols);
  return hipGetLastError();
}
