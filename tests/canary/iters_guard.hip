// Compiler canary for DESIGN.md §8 (ROCm 7.2, gfx950): the simple kernel of the Sierpinski
// family built WITHOUT the ITERS workaround's trip-count assumption. tests/test_compiler_canary.py
// compiles this file to gfx950 assembly only (it is never run: on a GPU the miscompiled kernel
// loops ~2^32 times for num_iterations == 0) and looks for the miscompile's signature: the
// uniform guard "num_iterations > 0" materialised as a 0/1 VGPR before the march loop and
// turned back into a lane mask by a compare inside the loop, where lanes that already left
// the march are inactive and get a 0 bit.
#ifndef FRM_CANARY_WITH_WORKAROUND  // the product's form, for the test's negative control
#define FRM_CANARY_NO_ITERS_ASSUME
#endif
#include "frm_render_kernels.h"

template __global__ void frm::render_simple<frm::kSierpinski, true>(frm::KernelArgs);
