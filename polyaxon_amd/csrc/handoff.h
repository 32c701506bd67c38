// In-launch hand-off of partial rows between the workgroups of one launch (the BatchNorm reduce + finalize, the LM
// bias column sums, the norm-weight partial sums): every producing workgroup writes its rows with agent-scope atomic
// stores (global_store ... sc1: coherent across the XCDs' L2s), every storing wave drains (s_waitcnt vmcnt(0)), a
// workgroup barrier, then ONE lane takes a relaxed agent-scope ticket; the workgroup whose ticket is last reads every
// row with agent-scope atomic loads (global_load ... sc1).  No buffer_wbl2 / buffer_inv: on gfx950 an agent release
// fence writes back the XCD's whole L2 and an acquire invalidates it, per workgroup (~1000 per launch).
//
// HARDWARE ASSUMPTION (not a C++/HIP memory-model guarantee): relaxed atomics carry no synchronises-with edge, so the
// reads being current relies on gfx950's sc1 stores reaching the coherence point before the waited-for vmcnt
// retires them and on sc1 loads bypassing the reading CU's L1 -- the "valid forms" measured for this chip
// (MI355X_MICROARCH.md, Workgroup dispatch / inter-workgroup visibility, first table row), and on the compiler not
// moving those loads above the barrier that follows the ticket.  tests/test_gpu_bn.py
// ::test_fence_free_handoff_stress checks it under load (hundreds of back-to-back launches, grids larger than the CU
// count, bitwise against the two-launch path).  Build with PLX_HANDOFF_FENCES=1 (ops/_native.py adds
// -DPLX_HANDOFF_FENCES=1) to restore the release / acquire fences of the architected recipe.
#pragma once

#ifndef PLX_HANDOFF_FENCES
#define PLX_HANDOFF_FENCES 0
#endif

// the signalling lane, after its workgroup's barrier and before the ticket add
__device__ __forceinline__ void plx_handoff_release() {
#if PLX_HANDOFF_FENCES
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // keep the fence's own wait (the compiler may drop it)
#endif
}

// the lane whose ticket was last, before the workgroup barrier that precedes the reads
__device__ __forceinline__ void plx_handoff_acquire() {
#if PLX_HANDOFF_FENCES
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
}
