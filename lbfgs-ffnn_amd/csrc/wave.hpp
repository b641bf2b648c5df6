// Wavefront (64-lane) primitives shared by the kernels.
//
// wave_sum_f64: fixed-order fp64 reduction through DPP lane moves (quad_perm, row_half_mirror,
// row_mirror, row_bcast15/31) — VALU moves instead of the ds_bpermute round trips a __shfl_xor
// butterfly costs (each a trip through the LDS crossbar). The sum lands in lane 63 and is broadcast
// with v_readlane, so every lane returns the same value. Deterministic: the addition tree is fixed.
// lane_f64: v_readlane of a wave-uniform lane index (the two-loop recurrences' per-step scalar).
#pragma once

#include <hip/hip_runtime.h>

namespace lbf {

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROW_MASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROW_MASK, 0xF, false);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double lane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double wave_sum_f64(double v) {
  v += dpp_f64<0xB1, 0xF>(v);  // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E, 0xF>(v);  // quad_perm [2,3,0,1]: quad sums
  v += dpp_f64<0x141, 0xF>(v); // row_half_mirror: 8-lane sums
  v += dpp_f64<0x140, 0xF>(v); // row_mirror: 16-lane row sums
  v += dpp_f64<0x142, 0xA>(v); // row_bcast15 into rows 1, 3
  v += dpp_f64<0x143, 0xC>(v); // row_bcast31 into rows 2, 3: lane 63 holds the total
  return lane_f64(v, 63);
}

// Workgroup barrier that orders LDS only. __syncthreads() carries a workgroup-scope release, which on
// gfx950 means s_waitcnt vmcnt(0): every global store the wave has in flight must be acknowledged
// (~1 us) before the barrier. Where no thread reads, after the barrier, global memory written before
// it by another thread of the block, the LDS wait is all the barrier has to order.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The speculative chain's abort flag (null: never aborted), requested as a vector load (an agent-scope
// relaxed atomic load is a global_load, counted by vmcnt). A kernel that tests it only once its first loads
// are in flight then does not wait for it in front of them; a scalar load of the flag would be covered by the
// kernel's first lgkmcnt wait for its arguments. Test it wave-uniformly: aborted(flag).
__device__ __forceinline__ int abort_flag(const int *p) {
  return p ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
}
__device__ __forceinline__ bool aborted(int flag) { return __builtin_amdgcn_readfirstlane(flag) != 0; }

} // namespace lbf
