// Compiler canary for DESIGN.md §8 (ROCm 7.2, gfx950): the simple kernel of the Sierpinski
// family built WITHOUT the ITERS workaround's trip-count assumption (csrc/frm_scene.h
// iterations<>). tests/test_compiler_canary.py compiles this file to gfx950 assembly only
// (it is never run: on a GPU the miscompiled kernel loops ~2^32 times for
// num_iterations == 0) and looks for the miscompile's signature: the uniform guard
// "num_iterations > 0" materialised as a 0/1 VGPR before the march loop and turned back into
// a lane mask by a compare inside the loop, where lanes that already left the march are
// inactive and get a 0 bit.
#include "frm_render_kernels.h"

#ifndef FRM_CANARY_WITH_WORKAROUND  // without it: the product's form, the test's negative control
// iterations<true> without FRM_ASSUME(n >= 1): the guard "n > 0" is back in every fold loop
// (an explicit specialization, declared before the instantiation below is the first use)
namespace frm {
template <>
FRM_HD uint32_t iterations<true>(uint32_t n) {
  return n;
}
}  // namespace frm
#endif

template __global__ void frm::render_simple<frm::kSierpinski, true>(frm::KernelArgs);
