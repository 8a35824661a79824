// xcc_map.hip -- where the dispatcher places blocks: per launch, the XCD (HW_REG_XCC_ID) of every block,
// for a sequence like the headline's (a 2,070-block forward, then a 209-block backward, then a 261-block
// sums launch), eager and graph-replayed.  Prints per launch: block 0's XCD and whether every block b sat
// on (xcd(0) + b) % 8 (round-robin).  A study tool (speed-only placement facts), not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void xcc_kernel(int* out) {
  if (threadIdx.x == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    out[blockIdx.x] = (int)(x & 0xF);
  }
}

#define CK(e) do { hipError_t r = (e); if (r != hipSuccess) { printf("HIP error %d line %d\n", (int)r, __LINE__); return 1; } } while (0)

int main() {
  const int grids[3] = {2070, 209, 261};
  const int reps = 4;
  int* d;
  CK(hipMalloc(&d, sizeof(int) * 3 * reps * 4096));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  auto launch_all = [&](int base) {
    for (int r = 0; r < reps; ++r)
      for (int k = 0; k < 3; ++k)
        hipLaunchKernelGGL(xcc_kernel, dim3(grids[k]), dim3(512), 0, s, d + (base + r * 3 + k) * 4096);
  };
  auto report = [&](const char* tag) -> int {
    std::vector<int> h(3 * reps * 4096);
    CK(hipMemcpy(h.data(), d, h.size() * sizeof(int), hipMemcpyDeviceToHost));
    for (int r = 0; r < reps; ++r)
      for (int k = 0; k < 3; ++k) {
        const int* o = h.data() + (r * 3 + k) * 4096;
        int rr = 1;
        for (int b = 0; b < grids[k]; ++b) rr &= o[b] == (o[0] + b) % 8;
        printf("%s rep %d launch %d (%d blocks): block0 xcd %d, round-robin %s, last block xcd %d\n", tag, r, k,
               grids[k], o[0], rr ? "yes" : "NO", o[grids[k] - 1]);
      }
    return 0;
  };
  launch_all(0);
  CK(hipStreamSynchronize(s));
  if (report("eager")) return 1;
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  launch_all(0);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) {
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    char tag[32];
    snprintf(tag, sizeof tag, "graph%d", i);
    if (report(tag)) return 1;
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipFree(d));
  return 0;
}
