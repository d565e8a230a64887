// Minimal HIP reproducer for the round-2/3 single-graph capture crash, no torch involved.
//
// The torch-level bisection (probe/capture_bisect.py) pinned the segfault inside
// hipStreamEndCapture on a SECOND-LEVEL fork: capture stream s0 -> depth_net's stream s1 (forked from s0) -> its
// filter-gradient stream s2 (forked from s1), joined back s2 -> s1 -> s0.  This program builds exactly that
// topology with plain HIP calls and reports, per variant, whether capture / instantiate / replay succeed and
// whether the replayed result is right:
//   1  one second-level fork and join
//   2  40 rounds of "kernel on s1, event on s1, s2 waits, kernel on s2" (a backward with per-layer forks), one join
//   3  as 2, every fork event destroyed right after its wait (torch's temporary events in Stream.wait_stream)
//   4  as 2, ONE event re-recorded for every fork (event reuse inside the capture)
//   5  as 2, s2 joined straight into s0 (skipping s1) and s1 joined into s0 afterwards
//   6  as 2 with a first-level fork of s3 from s0 as well (two side branches of the origin, one of them nested)
// Usage: capture_fork2 <variant>   (one variant per process, so a crash names its variant)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::printf("variant %d: %s failed: %s\n", variant, #x, hipGetErrorString(e_));    \
      std::fflush(stdout);                                                               \
      return 2;                                                                          \
    }                                                                                    \
  } while (0)

__global__ void add_kernel(float* p, int n, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += v;
}

static void add(hipStream_t s, float* p, int n, float v) {
  hipLaunchKernelGGL(add_kernel, dim3((n + 255) / 256), dim3(256), 0, s, p, n, v);
}

int main(int argc, char** argv) {
  const int variant = argc > 1 ? std::atoi(argv[1]) : 1;
  const int n = 1 << 16;
  const int rounds = variant == 1 ? 1 : 40;
  float *a, *b, *c;
  CK(hipMalloc(&a, n * sizeof(float)));
  CK(hipMalloc(&b, n * sizeof(float)));
  CK(hipMalloc(&c, n * sizeof(float)));
  CK(hipMemset(a, 0, n * sizeof(float)));
  CK(hipMemset(b, 0, n * sizeof(float)));
  CK(hipMemset(c, 0, n * sizeof(float)));
  hipStream_t s0, s1, s2, s3;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
  std::vector<hipEvent_t> keep;
  auto ev = [&](hipEvent_t* e) { return hipEventCreateWithFlags(e, hipEventDisableTiming); };
  hipEvent_t reuse;
  CK(ev(&reuse));

  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
  add(s0, a, n, 1.f);
  hipEvent_t e0;
  CK(ev(&e0));
  keep.push_back(e0);
  CK(hipEventRecord(e0, s0));
  CK(hipStreamWaitEvent(s1, e0, 0));         // first-level fork: s1 from the origin
  if (variant == 6) {
    hipEvent_t e3;
    CK(ev(&e3));
    keep.push_back(e3);
    CK(hipEventRecord(e3, s0));
    CK(hipStreamWaitEvent(s3, e3, 0));       // a second first-level branch
    add(s3, c, n, 5.f);
  }
  for (int r = 0; r < rounds; ++r) {
    add(s1, a, n, 1.f);
    hipEvent_t e;
    if (variant == 4) {
      e = reuse;
    } else {
      CK(ev(&e));
    }
    CK(hipEventRecord(e, s1));
    CK(hipStreamWaitEvent(s2, e, 0));        // second-level fork: s2 from s1
    if (variant == 3) CK(hipEventDestroy(e));
    else if (variant != 4) keep.push_back(e);
    add(s2, b, n, 2.f);
  }
  hipEvent_t j2, j1;
  CK(ev(&j2));
  CK(ev(&j1));
  keep.push_back(j2);
  keep.push_back(j1);
  if (variant == 5) {
    CK(hipEventRecord(j2, s2));
    CK(hipStreamWaitEvent(s0, j2, 0));       // s2 -> origin directly
    CK(hipEventRecord(j1, s1));
    CK(hipStreamWaitEvent(s0, j1, 0));
  } else {
    CK(hipEventRecord(j2, s2));
    CK(hipStreamWaitEvent(s1, j2, 0));       // s2 -> s1
    CK(hipEventRecord(j1, s1));
    CK(hipStreamWaitEvent(s0, j1, 0));       // s1 -> origin
  }
  if (variant == 6) {
    hipEvent_t j3;
    CK(ev(&j3));
    keep.push_back(j3);
    CK(hipEventRecord(j3, s3));
    CK(hipStreamWaitEvent(s0, j3, 0));
  }
  add(s0, a, n, 1.f);
  hipGraph_t g;
  std::printf("variant %d: ending capture ...\n", variant);
  std::fflush(stdout);
  CK(hipStreamEndCapture(s0, &g));
  size_t nodes = 0;
  CK(hipGraphGetNodes(g, nullptr, &nodes));
  hipGraphExec_t x;
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  for (int it = 0; it < 3; ++it) CK(hipGraphLaunch(x, s0));
  CK(hipStreamSynchronize(s0));
  float ha = 0, hb = 0, hc = 0;
  CK(hipMemcpy(&ha, a + n - 1, sizeof(float), hipMemcpyDeviceToHost));
  CK(hipMemcpy(&hb, b + n - 1, sizeof(float), hipMemcpyDeviceToHost));
  CK(hipMemcpy(&hc, c + n - 1, sizeof(float), hipMemcpyDeviceToHost));
  const float wa = 3.f * (2 + rounds), wb = 3.f * 2 * rounds, wc = variant == 6 ? 15.f : 0.f;
  const bool ok = ha == wa && hb == wb && hc == wc;
  std::printf("variant %d: capture ok, %zu nodes, 3 replays: a=%g (want %g) b=%g (want %g) c=%g (want %g) -> %s\n",
              variant, nodes, ha, wa, hb, wb, hc, wc, ok ? "PASS" : "WRONG");
  CK(hipGraphExecDestroy(x));
  CK(hipGraphDestroy(g));
  for (hipEvent_t e : keep) CK(hipEventDestroy(e));
  CK(hipEventDestroy(reuse));
  return ok ? 0 : 1;
}
