// Launcher of gpk_kzz.hip (the 16-column K_ZZ factor + the L^{-1} kernel), for the C-ABI shim.
#pragma once
#include <hip/hip_runtime.h>

struct GpkKzzArgs;
int gpk_launch_kzz16(const GpkKzzArgs& a, hipStream_t stream);
