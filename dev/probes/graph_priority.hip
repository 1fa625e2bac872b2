// A latency-bound chain (K kernels of 256 one-per-CU workgroups, ~6 us each) next to a
// throughput-bound branch (big grids that fill every CU) in one graph: how long does the
// chain take, with and without node priorities (hipLaunchAttributePriority +
// hipGraphInstantiateFlagUseNodePriority), and eagerly on two streams of different priority.
// hipcc --offload-arch=gfx950 -O2 graph_priority.hip -o dev/bin/graph_priority
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void chain_k(long long cycles, long long* stamp, int k) {
  extern __shared__ char lds[];
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {}
  lds[threadIdx.x] = 1;
  if (blockIdx.x == 0 && threadIdx.x == 0) stamp[k] = wall_clock64() + lds[0] - 1;
}
__global__ void big_k(long long cycles, long long* stamp) {
  extern __shared__ char lds[];
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {}
  lds[threadIdx.x] = 1;
  if (blockIdx.x == 0 && threadIdx.x == 0) stamp[1000] = wall_clock64() + lds[0] - 1;
}
__global__ void start_k(long long* stamp) { if (threadIdx.x == 0) stamp[999] = wall_clock64(); }

int main() {
  const int K = 32, NB = 12;
  long long* stamp; CK(hipMalloc(&stamp, 8192 * 8));
  int khz = 100000;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  long long c_chain = (long long)khz * 6 / 1000, c_big = (long long)khz * 20 / 1000;
  CK(hipFuncSetAttribute((const void*)chain_k, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024));
  CK(hipFuncSetAttribute((const void*)big_k, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  printf("priority range least %d greatest %d; chain %d x ~6 us (256 WG, 100 KB LDS), big %d x ~20 us x 4 rounds\n",
         lo, hi, K, NB);

  auto build = [&](int mode) -> hipGraphExec_t {   // 0 chain only, 1 big only, 2 both, 3 both + priority
    hipGraph_t g; (void)hipGraphCreate(&g, 0);
    hipGraphNode_t root; (void)hipGraphAddEmptyNode(&root, g, nullptr, 0);
    hipGraphNode_t st; hipKernelNodeParams sp = {};
    void* sargs[] = {&stamp};
    sp.func = (void*)start_k; sp.gridDim = dim3(1); sp.blockDim = dim3(64); sp.kernelParams = sargs;
    (void)hipGraphAddKernelNode(&st, g, &root, 1, &sp);
    std::vector<std::vector<void*>> keep;
    static int ks[64];
    if (mode != 1) {
      hipGraphNode_t prev = st;
      for (int k = 0; k < K; ++k) {
        ks[k] = k;
        static void* a[64][3];
        a[k][0] = &c_chain; a[k][1] = &stamp; a[k][2] = &ks[k];
        hipKernelNodeParams kp = {};
        kp.func = (void*)chain_k; kp.gridDim = dim3(256); kp.blockDim = dim3(256); kp.sharedMemBytes = 100 * 1024;
        kp.kernelParams = a[k];
        hipGraphNode_t n; (void)hipGraphAddKernelNode(&n, g, &prev, 1, &kp);
        if (mode == 3) {
          hipKernelNodeAttrValue v = {};
          v.priority = hi;
          hipError_t e = hipGraphKernelNodeSetAttribute(n, hipKernelNodeAttributePriority, &v);
          if (e != hipSuccess && k == 0) printf("  set priority: %s\n", hipGetErrorString(e));
        }
        prev = n;
      }
    }
    if (mode != 0) {
      hipGraphNode_t prev = st;
      static void* b[2];
      b[0] = &c_big; b[1] = &stamp;
      for (int k = 0; k < NB; ++k) {
        hipKernelNodeParams kp = {};
        kp.func = (void*)big_k; kp.gridDim = dim3(256 * 2 * 4); kp.blockDim = dim3(256); kp.sharedMemBytes = 64 * 1024;
        kp.kernelParams = b;
        hipGraphNode_t n; (void)hipGraphAddKernelNode(&n, g, &prev, 1, &kp);
        prev = n;
      }
    }
    hipGraphExec_t ex;
    hipError_t e = hipGraphInstantiateWithFlags(&ex, g, mode == 3 ? hipGraphInstantiateFlagUseNodePriority : 0);
    if (e != hipSuccess) { printf("instantiate: %s\n", hipGetErrorString(e)); return nullptr; }
    return ex;
  };
  hipStream_t s0; CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  const char* names[] = {"chain alone", "big alone", "both", "both, chain nodes high priority"};
  for (int mode = 0; mode < 4; ++mode) {
    hipGraphExec_t ex = build(mode);
    if (!ex) continue;
    double best_all = 1e30, best_chain = 1e30;
    for (int r = 0; r < 4; ++r) {
      hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
      (void)hipEventRecord(a, s0);
      (void)hipGraphLaunch(ex, s0);
      (void)hipEventRecord(b, s0);
      (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b);
      std::vector<long long> h(1001);
      (void)hipMemcpy(h.data(), stamp, 1001 * 8, hipMemcpyDeviceToHost);
      const double chain_us = (h[K - 1] - h[999]) * 1000.0 / khz;
      if (r) { best_all = std::min(best_all, (double)ms * 1000.0); if (mode != 1) best_chain = std::min(best_chain, chain_us); }
    }
    printf("%-34s total %8.1f us   chain done after %8.1f us\n", names[mode], best_all, mode == 1 ? 0.0 : best_chain);
  }
  // eager: chain on a high-priority stream, big on a low-priority one
  for (int pr = 0; pr < 2; ++pr) {
    hipStream_t sc, sb;
    CK(hipStreamCreateWithPriority(&sc, hipStreamNonBlocking, pr ? hi : lo));
    CK(hipStreamCreateWithPriority(&sb, hipStreamNonBlocking, lo));
    double best = 1e30, best_all = 1e30;
    for (int r = 0; r < 4; ++r) {
      hipEvent_t a, b, j; (void)hipEventCreate(&a); (void)hipEventCreate(&b); (void)hipEventCreate(&j);
      (void)hipEventRecord(a, sc);
      (void)hipStreamWaitEvent(sb, a, 0);
      hipLaunchKernelGGL(start_k, dim3(1), dim3(64), 0, sc, stamp);
      for (int k = 0; k < NB; ++k) hipLaunchKernelGGL(big_k, dim3(2048), dim3(256), 64 * 1024, sb, c_big, stamp);
      for (int k = 0; k < K; ++k) hipLaunchKernelGGL(chain_k, dim3(256), dim3(256), 100 * 1024, sc, c_chain, stamp, k);
      (void)hipEventRecord(j, sb);
      (void)hipStreamWaitEvent(sc, j, 0);
      (void)hipEventRecord(b, sc);
      (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b);
      std::vector<long long> h(1001);
      (void)hipMemcpy(h.data(), stamp, 1001 * 8, hipMemcpyDeviceToHost);
      if (r) { best = std::min(best, (h[K - 1] - h[999]) * 1000.0 / khz); best_all = std::min(best_all, (double)ms * 1000.0); }
    }
    printf("eager two streams, chain %-9s total %8.1f us   chain done after %8.1f us\n", pr ? "high prio" : "same prio",
           best_all, best);
  }
  return 0;
}
