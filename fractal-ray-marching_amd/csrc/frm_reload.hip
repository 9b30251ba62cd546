// frm_reload.hip — runtime kernel reload: the reference's shader hot
// reload (`r` key, graphics.rs:39-48 -> reloadable_graphics.rs:15-52: read fragment.wgsl
// from disk, rebuild the pipeline, print the error and keep the old pipeline on failure).
//
// Here the edited sources are a copy of this package's csrc/ headers: frm_render_kernels.h
// (the render kernels) and the headers it includes (frm_scene.h: scenes and distance
// estimators, frm_math.h: builtins, shading constants, ...). hiprtc compiles them for the
// device's own architecture with the same math flags as the ahead-of-time build; the code
// object is loaded with hipModuleLoadData and every later render of the context launches
// its kernels through hipModuleLaunchKernel (frm_kernels.hip launchers).
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdio.h>
#include <sys/stat.h>

#include <algorithm>
#include <string>
#include <vector>

#include "frm_internal.h"

#if !defined(FRM_RELOAD_MLLVM) || !defined(FRM_RELOAD_MARCH_WAVES)
#error "built by the Makefile, which passes the render kernels' code-generation options (SCHED_MLLVM, MARCH_WAVES)"
#endif

#ifndef FRM_INCLUDE_DIR  // this package's include/ (frm.h), set by the Makefile
#define FRM_INCLUDE_DIR ""
#endif

namespace frm {
namespace {

// hiprtc puts the fixed-width types in __hip_internal and has no <stdint.h>.
const char kSource[] =
    "typedef __hip_internal::uint8_t uint8_t;\n"
    "typedef __hip_internal::uint16_t uint16_t;\n"
    "typedef __hip_internal::uint32_t uint32_t;\n"
    "typedef __hip_internal::uint64_t uint64_t;\n"
    "typedef __hip_internal::int32_t int32_t;\n"
    "typedef __hip_internal::int64_t int64_t;\n"
    "#include \"frm_render_kernels.h\"\n";

bool is_file(const std::string& p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

std::string kernel_name(int kind, uint32_t fam, bool iters) {
  const std::string f = std::to_string(fam) + "u";
  const char* it = iters ? "true" : "false";
  if (kind == 0) return "frm::render_simple<" + f + ", " + it + ">";
  if (kind == 1) return "frm::march_persistent<" + f + ", " + it + ">";
  return "frm::shade_pass<" + f + ">";
}

}  // namespace

int compile_reloaded(const char* dir, int device, ReloadedKernels** out, std::string* log) {
  *out = nullptr;
  const std::string d(dir);
  if (!is_file(d + "/frm_render_kernels.h")) {
    *log = "no frm_render_kernels.h in " + d;
    return FRM_ERR_INVALID_ARGUMENT;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    *log = "hipGetDeviceProperties failed";
    return FRM_ERR_HIP;
  }
  std::string arch = std::string("--offload-arch=") + prop.gcnArchName;
  const size_t colon = arch.find(':');  // "gfx950:sramecc+:xnack-" -> "gfx950"
  if (colon != std::string::npos) arch.resize(colon);
  // the AOT build's code-generation options for the render kernels, passed in by the Makefile from
  // the variables that build frm_kernels.o (SCHED_MLLVM, MARCH_WAVES): no SLP vectorisation into
  // packed f32 ops, the register-pressure trackers, wave-uniform branches left unstructurized, and
  // the march kernel's waves per SIMD, so a reloaded kernel has the built-in one's occupancy
  std::vector<std::string> opts = {arch, "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                                   "-fno-slp-vectorize",
                                   "-DFRM_MARCH_WAVES_PER_SIMD=" + std::to_string(FRM_RELOAD_MARCH_WAVES), "-I" + d};
  {
    const std::string mllvm(FRM_RELOAD_MLLVM);
    for (size_t i = 0; i < mllvm.size();) {
      const size_t j = std::min(mllvm.find(' ', i), mllvm.size());
      if (j > i) {
        opts.push_back("-mllvm");
        opts.push_back(mllvm.substr(i, j - i));
      }
      i = j + 1;
    }
  }
  // frm.h: next to the sources, in ../include or ../../include of them, or this build's
  for (const std::string& inc : {d + "/../include", d + "/../../include", std::string(FRM_INCLUDE_DIR)})
    if (!inc.empty() && is_file(inc + "/frm.h")) opts.push_back("-I" + inc);

  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, kSource, "frm_reload.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
    *log = "hiprtcCreateProgram failed";
    return FRM_ERR_COMPILE;
  }
  std::vector<std::string> names;
  for (uint32_t f = 0; f < kNumFamilies; ++f) {
    for (int it = 0; it < 2; ++it) {
      names.push_back(kernel_name(0, f, it));
      names.push_back(kernel_name(1, f, it));
    }
    names.push_back(kernel_name(2, f, false));
  }
  for (const std::string& n : names) hiprtcAddNameExpression(prog, n.c_str());
  std::vector<const char*> argv;
  for (const std::string& o : opts) argv.push_back(o.c_str());
  const hiprtcResult rc = hiprtcCompileProgram(prog, (int)argv.size(), argv.data());
  size_t log_size = 0;
  hiprtcGetProgramLogSize(prog, &log_size);
  std::string compiler_log(log_size, '\0');
  if (log_size) hiprtcGetProgramLog(prog, &compiler_log[0]);
  if (rc != HIPRTC_SUCCESS) {
    *log = std::string(hiprtcGetErrorString(rc)) + ":\n" + compiler_log;
    hiprtcDestroyProgram(&prog);
    return FRM_ERR_COMPILE;
  }
  size_t code_size = 0;
  hiprtcGetCodeSize(prog, &code_size);
  std::vector<char> code(code_size);
  hiprtcGetCode(prog, code.data());

  ReloadedKernels* rk = new ReloadedKernels();
  int status = FRM_OK;
  if (hipModuleLoadData(&rk->module, code.data()) != hipSuccess) {
    *log = "hipModuleLoadData failed";
    status = FRM_ERR_HIP;
  }
  for (uint32_t f = 0; f < kNumFamilies && status == FRM_OK; ++f) {
    for (int it = 0; it < 2 && status == FRM_OK; ++it) {
      for (int kind = 0; kind < 2 && status == FRM_OK; ++kind) {
        const char* lowered = nullptr;
        hipFunction_t fn = nullptr;
        if (hiprtcGetLoweredName(prog, kernel_name(kind, f, it).c_str(), &lowered) != HIPRTC_SUCCESS ||
            hipModuleGetFunction(&fn, rk->module, lowered) != hipSuccess) {
          *log = "kernel not found: " + kernel_name(kind, f, it);
          status = FRM_ERR_COMPILE;
        } else if (kind == 0) {
          rk->simple[f][it] = fn;
        } else {
          rk->persistent[f][it] = fn;
          int n = 0;
          (void)hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kMarchBlock, 0);
          rk->persistent_blocks_per_cu[f][it] = n > 0 ? n : 1;
        }
      }
    }
    const char* lowered = nullptr;
    if (status == FRM_OK && (hiprtcGetLoweredName(prog, kernel_name(2, f, false).c_str(), &lowered) != HIPRTC_SUCCESS ||
                             hipModuleGetFunction(&rk->shade[f], rk->module, lowered) != hipSuccess)) {
      *log = "kernel not found: " + kernel_name(2, f, false);
      status = FRM_ERR_COMPILE;
    }
  }
  hiprtcDestroyProgram(&prog);
  if (status != FRM_OK) {
    unload_reloaded(rk);
    return status;
  }
  *log = compiler_log;  // warnings, if any
  *out = rk;
  return FRM_OK;
}

void unload_reloaded(ReloadedKernels* rk) {
  if (!rk) return;
  if (rk->module) (void)hipModuleUnload(rk->module);
  delete rk;
}

}  // namespace frm
