// Probe: can a kernel inside a captured HIP graph be bracketed by event-record nodes
// (hipEventRecordWithFlags(..., hipEventRecordExternal) during stream capture), and do the
// events then time each replay?  Also tries hipGraphAddEventRecordNode on the captured graph.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(float* p, int n, int iters) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = p[i];
  for (int k = 0; k < iters; ++k) v = v * 1.0000001f + 1e-7f;
  p[i] = v;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); } } while (0)

int main() {
  const int n = 1 << 20;
  float* d;
  CK(hipMalloc(&d, n * 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (unsigned flags : {(unsigned)hipEventDefault, (unsigned)hipEventBlockingSync}) {
    hipEvent_t e0, e1;
    CK(hipEventCreateWithFlags(&e0, flags));
    CK(hipEventCreateWithFlags(&e1, flags));
    hipGraph_t g;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    hipLaunchKernelGGL(spin, dim3(n / 256), dim3(256), 0, s, d, n, 2000);
    hipError_t r0 = hipEventRecordWithFlags(e0, s, hipEventRecordExternal);
    hipLaunchKernelGGL(spin, dim3(n / 256), dim3(256), 0, s, d, n, 20000);
    hipError_t r1 = hipEventRecordWithFlags(e1, s, hipEventRecordExternal);
    hipLaunchKernelGGL(spin, dim3(n / 256), dim3(256), 0, s, d, n, 2000);
    CK(hipStreamEndCapture(s, &g));
    printf("flags %u: record external during capture: %s / %s, last error %s\n", flags,
           hipGetErrorString(r0), hipGetErrorString(r1), hipGetErrorString(hipGetLastError()));
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      float ms = -1;
      hipError_t q = hipEventElapsedTime(&ms, e0, e1);
      printf("  replay %d: elapsed %s %.4f ms\n", rep, hipGetErrorString(q), ms);
    }
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    printf("  nodes %zu\n", nn);
  }
  // plain hipEventRecord inside a capture (how torch's fork/join records): allowed?
  {
    hipEvent_t e0;
    CK(hipEventCreate(&e0));
    hipGraph_t g;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    hipError_t r = hipEventRecord(e0, s);
    hipLaunchKernelGGL(spin, dim3(n / 256), dim3(256), 0, s, d, n, 10);
    CK(hipStreamEndCapture(s, &g));
    printf("plain record during capture: %s\n", hipGetErrorString(r));
  }
  printf("probe done\n");
  return 0;
}
