// Cost of cross-stream edges inside a captured hipGraph on MI355X: a chain of
// NK busy kernels on stream A (each ~T us on every CU), with F side-stream
// kernels forked off the chain (event record on A -> wait on B) and joined
// back (record on B -> wait on A) at evenly spaced points.  Prints the replay
// time per configuration; the difference to the plain chain is the edge cost.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t ck_ = (x); if (ck_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(ck_)); return 1; } } while (0)

__global__ void busy(float* out, int iters) {
  float v = threadIdx.x;
  for (int i = 0; i < iters; ++i) v = v * 0.999f + 0.5f;
  if (v == -1.f) out[blockIdx.x] = v;  // keep the loop
}

int run(int nk, int forks, int mode, int iters, float* buf, double* us) {
  // mode 0: fork + join per side kernel; 1: fork only (joined at the end); 2: join only (side forked at start)
  hipStream_t a, b, cap;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(4 * nk + 4);
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
  int ei = 0;
  CK(hipEventRecord(ev[ei], cap));
  CK(hipStreamWaitEvent(a, ev[ei], 0));
  CK(hipStreamWaitEvent(b, ev[ei], 0));
  ++ei;
  const int every = forks ? nk / (forks + 1) : nk + 1;
  for (int k = 0; k < nk; ++k) {
    hipLaunchKernelGGL(busy, dim3(256), dim3(256), 0, a, buf, iters);
    if (forks && (k + 1) % every == 0 && (k + 1) / every <= forks) {
      if (mode != 2) {
        CK(hipEventRecord(ev[ei], a));
        CK(hipStreamWaitEvent(b, ev[ei], 0));
        ++ei;
      }
      hipLaunchKernelGGL(busy, dim3(32), dim3(256), 0, b, buf, iters / 4);
      if (mode != 1) {
        CK(hipEventRecord(ev[ei], b));
        CK(hipStreamWaitEvent(a, ev[ei], 0));
        ++ei;
      }
    }
  }
  CK(hipEventRecord(ev[ei], a));
  CK(hipStreamWaitEvent(cap, ev[ei], 0));
  ++ei;
  CK(hipEventRecord(ev[ei], b));
  CK(hipStreamWaitEvent(cap, ev[ei], 0));
  ++ei;
  CK(hipStreamEndCapture(cap, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, cap));
  CK(hipStreamSynchronize(cap));
  const int reps = 20;
  auto t0 = std::chrono::high_resolution_clock::now();
  for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, cap));
  CK(hipStreamSynchronize(cap));
  auto t1 = std::chrono::high_resolution_clock::now();
  *us = std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  for (auto& e : ev) CK(hipEventDestroy(e));
  CK(hipStreamDestroy(a));
  CK(hipStreamDestroy(b));
  CK(hipStreamDestroy(cap));
  return 0;
}

int main() {
  float* buf;
  CK(hipMalloc(&buf, 1 << 20));
  const int nk = 40, iters = 4000;
  double base;
  if (run(nk, 0, 0, iters, buf, &base)) return 1;
  printf("chain of %d kernels: %.1f us per replay (%.2f us per kernel)\n", nk, base, base / nk);
  for (int mode = 0; mode < 3; ++mode)
    for (int f : {1, 4, 9}) {
      double t;
      if (run(nk, f, mode, iters, buf, &t)) return 1;
      const int edges = mode == 0 ? 2 * f : f;
      printf("mode %s forks %d: %.1f us (+%.1f us, %.2f us per edge)\n",
             mode == 0 ? "fork+join" : mode == 1 ? "fork-only" : "join-only", f, t, t - base, (t - base) / edges);
    }
  CK(hipFree(buf));
  return 0;
}
