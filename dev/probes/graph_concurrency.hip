// Does the HIP graph executor run independent branches concurrently?  Two chains of K
// spin kernels (one workgroup each, ~T us) as
//   A: two disconnected components (nodes added with hipGraphAddKernelNode)
//   B: A plus one empty root node both chains depend on
//   C: stream capture, chain 2 forked onto a second stream by events (fork + join)
//   D: the two chains as two graphs launched on two streams
//   S: one chain alone (reference)
// hipcc --offload-arch=gfx950 -O2 graph_concurrency.hip -o /tmp/gc && /tmp/gc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void spin(long long cycles, int* out) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {}
  if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

static float time_exec(hipGraphExec_t ex, hipStream_t s, int reps = 5) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  (void)hipGraphLaunch(ex, s);
  (void)hipStreamSynchronize(s);
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    (void)hipEventRecord(a, s);
    (void)hipGraphLaunch(ex, s);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  return best * 1000.f;
}

int main() {
  const int K = 20;
  int* out; CK(hipMalloc(&out, 4096));
  int rate_khz = 100000;
  (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
  long long cyc = (long long)rate_khz * 50 / 1000;   // ~50 us per kernel
  printf("wall clock %d kHz, %d kernels per chain, ~50 us each\n", rate_khz, K);
  void* args[] = {&cyc, &out};
  hipKernelNodeParams kp = {};
  kp.func = (void*)spin;
  kp.gridDim = dim3(1);
  kp.blockDim = dim3(64);
  kp.kernelParams = args;
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));

  auto chains = [&](bool root, int nchains) -> hipGraphExec_t {
    hipGraph_t g; (void)hipGraphCreate(&g, 0);
    hipGraphNode_t r = nullptr;
    if (root) (void)hipGraphAddEmptyNode(&r, g, nullptr, 0);
    for (int c = 0; c < nchains; ++c) {
      hipGraphNode_t prev = r;
      for (int k = 0; k < K; ++k) {
        hipGraphNode_t n;
        (void)hipGraphAddKernelNode(&n, g, prev ? &prev : nullptr, prev ? 1 : 0, &kp);
        prev = n;
      }
    }
    hipGraphExec_t ex; (void)hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    return ex;
  };
  printf("S one chain          %8.1f us\n", time_exec(chains(false, 1), s0));
  printf("A two components     %8.1f us\n", time_exec(chains(false, 2), s0));
  printf("B two + root         %8.1f us\n", time_exec(chains(true, 2), s0));

  // interleaved creation order (chain 1 node k, chain 2 node k, ...)
  {
    hipGraph_t g; (void)hipGraphCreate(&g, 0);
    hipGraphNode_t prev[2] = {nullptr, nullptr};
    for (int k = 0; k < K; ++k)
      for (int c = 0; c < 2; ++c) {
        hipGraphNode_t n;
        (void)hipGraphAddKernelNode(&n, g, prev[c] ? &prev[c] : nullptr, prev[c] ? 1 : 0, &kp);
        prev[c] = n;
      }
    hipGraphExec_t ex; (void)hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    printf("A' interleaved order %8.1f us\n", time_exec(ex, s0));
  }

  // C: stream capture with fork / join
  {
    hipEvent_t f, j;
    CK(hipEventCreateWithFlags(&f, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
    hipGraph_t g;
    CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
    CK(hipEventRecord(f, s0));
    CK(hipStreamWaitEvent(s1, f, 0));
    for (int k = 0; k < K; ++k) {
      hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s0, cyc, out);
      hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s1, cyc, out);
    }
    CK(hipEventRecord(j, s1));
    CK(hipStreamWaitEvent(s0, j, 0));
    CK(hipStreamEndCapture(s0, &g));
    hipGraphExec_t ex; CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    printf("C captured fork/join %8.1f us\n", time_exec(ex, s0));
  }
  // D: two graphs, two streams
  {
    hipGraphExec_t e1 = chains(false, 1), e2 = chains(false, 1);
    hipEvent_t a, b, j;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b); (void)hipEventCreate(&j);
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
      (void)hipEventRecord(a, s0);
      (void)hipStreamWaitEvent(s1, a, 0);
      (void)hipGraphLaunch(e1, s0);
      (void)hipGraphLaunch(e2, s1);
      (void)hipEventRecord(j, s1);
      (void)hipStreamWaitEvent(s0, j, 0);
      (void)hipEventRecord(b, s0);
      (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b);
      if (r && ms < best) best = ms;
    }
    printf("D two graphs/streams %8.1f us\n", best * 1000.f);
  }
  // E: plain stream launches on two streams (no graph)
  {
    hipEvent_t a, b, j;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b); (void)hipEventCreate(&j);
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
      (void)hipEventRecord(a, s0);
      (void)hipStreamWaitEvent(s1, a, 0);
      for (int k = 0; k < K; ++k) {
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s0, cyc, out);
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s1, cyc, out);
      }
      (void)hipEventRecord(j, s1);
      (void)hipStreamWaitEvent(s0, j, 0);
      (void)hipEventRecord(b, s0);
      (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b);
      if (r && ms < best) best = ms;
    }
    printf("E eager two streams  %8.1f us\n", best * 1000.f);
  }
  return 0;
}
