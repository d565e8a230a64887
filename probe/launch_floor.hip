// Launch-floor probe: back-to-back dependent tiny kernels on one stream, plain launches vs hipGraph
// replay (diagnostic for the per-kernel cost that bounds the small layers).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <chrono>

__global__ void tiny(float* p, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5f + 1.0f;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
  const int K = 200;
  float* d; CK(hipMalloc(&d, 64 << 20));
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int blocks : {1, 64, 1024}) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(a, s));
      for (int i = 0; i < K; ++i) hipLaunchKernelGGL(tiny, dim3(blocks), dim3(256), 0, s, d, blocks * 256);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (rep) printf("stream  blocks %5d: %.2f us/kernel\n", blocks, ms * 1e3 / K);
    }
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(tiny, dim3(blocks), dim3(256), 0, s, d, blocks * 256);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (rep) printf("graph   blocks %5d: %.2f us/kernel\n", blocks, ms * 1e3 / K);
    }
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
  }
  // a large-footprint writer before each tiny kernel: does the boundary cost grow with dirty L2 data?
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipEventRecord(a, s));
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(tiny, dim3(4096), dim3(256), 0, s, d, 4096 * 256);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (rep) printf("stream 4 MB writers: %.2f us/kernel\n", ms * 1e3 / K);
  }
  return 0;
}
