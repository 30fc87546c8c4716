// probe: cost of an in-launch all-block hop on MI355X for G = 16 .. 256 resident blocks
// (one block per CU), three counter layouts, 200 hops per launch, bounded spins.
//   flat : every block adds 1 to ONE counter, one lane per block polls it
//   xcd  : every block adds to its XCD's counter; the XCD's last arriver (told by the value
//          its add returned) adds to the global counter; pollers poll the global counter
//   xcdf : as xcd, and the global last arriver stores the hop number into 8 per-XCD flag
//          lines; pollers poll their XCD's flag
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(1))) unsigned gu32;
#define RLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT
__device__ int xcc() { unsigned x; asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x)); return x & 7; }
__device__ bool spin(gu32* w, unsigned target, gu32* abort_w) {
  const unsigned long long t0 = wall_clock64();
  while (__hip_atomic_load(w, RLX) < target) {
    if (__hip_atomic_load(abort_w, RLX)) return false;
    if (wall_clock64() - t0 > 100000000ull) { __hip_atomic_store(abort_w, 1u, RLX); return false; }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}
// ctl: [0] global counter, [1] abort, [32 + 32 x] per-XCD counters, [320 + 32 x] flags,
// [600 + x] per-XCD block counts (census)
__global__ void hop_kernel(unsigned* ctl, int mode, int hops, unsigned long long* out) {
  __shared__ int ok;
  gu32* c = (gu32*)ctl;
  const int x = xcc();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(c + 600 + x, 1u, RLX);
  // census barrier (flat)
  if (threadIdx.x == 0) { __hip_atomic_fetch_add(c + 2, 1u, RLX); ok = spin(c + 2, gridDim.x, c + 1); }
  __syncthreads();
  if (!ok) return;
  unsigned nact = 0, nx = __hip_atomic_load(c + 600 + x, RLX);
  for (int i = 0; i < 8; ++i) nact += __hip_atomic_load(c + 600 + i, RLX) > 0;
  const unsigned long long t0 = wall_clock64();
  for (int h = 0; h < hops; ++h) {
    __syncthreads();
    if (threadIdx.x == 0) {
      bool r = true;
      if (mode == 0) {
        __hip_atomic_fetch_add(c, 1u, RLX);
        r = spin(c, (unsigned)gridDim.x * (h + 1), c + 1);
      } else {
        const unsigned old = __hip_atomic_fetch_add(c + 32 + 32 * x, 1u, RLX);
        if (old == nx * (h + 1) - 1) {  // last of this XCD
          const unsigned g = __hip_atomic_fetch_add(c, 1u, RLX);
          if (mode == 2 && g == nact * (h + 1) - 1)
            for (int i = 0; i < 8; ++i) __hip_atomic_store(c + 320 + 32 * i, (unsigned)(h + 1), RLX);
        }
        r = mode == 1 ? spin(c, nact * (h + 1), c + 1) : spin(c + 320 + 32 * x, h + 1, c + 1);
      }
      ok = r;
    }
    __syncthreads();
    if (!ok) return;
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = wall_clock64() - t0;
}
int main() {
  unsigned* ctl; unsigned long long* out;
  hipMalloc(&ctl, 4096); hipMalloc(&out, 8);
  const int hops = 200;
  for (int G : {16, 64, 128, 256}) {
    for (int mode = 0; mode < 3; ++mode) {
      double best = 1e30;
      for (int rep = 0; rep < 3; ++rep) {
        hipMemset(ctl, 0, 4096);
        hipLaunchKernelGGL(hop_kernel, dim3(G), dim3(256), 0, 0, ctl, mode, hops, out);
        unsigned long long t = 0; unsigned ab = 0;
        hipMemcpy(&t, out, 8, hipMemcpyDeviceToHost);
        hipMemcpy(&ab, ctl + 1, 4, hipMemcpyDeviceToHost);
        if (ab) { printf("G %d mode %d: TIMEOUT\n", G, mode); continue; }
        const double us = t / 100.0 / hops;  // 100 MHz wall clock
        if (us < best) best = us;
      }
      printf("G %3d %-5s %.2f us per hop\n", G, mode == 0 ? "flat" : mode == 1 ? "xcd" : "xcdf", best);
    }
  }
  return 0;
}
