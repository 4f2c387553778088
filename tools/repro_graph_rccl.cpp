// Torch-free reproducer of the round-5 graph-replay host fault (VERDICT r5
// item 1): HIP-graph captures and replays in one process, around a one-rank RCCL communicator
// whose all-reduces ran on one stream ("one") or two ("two"), destroyed ("...") or kept
// ("...-keep"); "...-big": 64 steps per graph (~320 nodes), launched on the null stream as
// torch's CUDAGraph.replay() does from the default current stream.  The Python reproducer (tools/repro_graph_rccl.py stream_close) segfaulted
// in hipGraphLaunch after the two-stream case; this program asks whether HIP + RCCL alone do.
//
//   hipcc --offload-arch=gfx950 -O2 tools/repro_graph_rccl.cpp -o tools/repro_graph_rccl \
//         -L/opt/rocm/lib -lrccl
//   ./tools/repro_graph_rccl two
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)
#define NK(x)                                                                        \
  do {                                                                               \
    ncclResult_t r_ = (x);                                                           \
    if (r_ != ncclSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_)); \
      exit(3);                                                                       \
    }                                                                                \
  } while (0)

__global__ void axpb(float* y, const float* x, float a, float b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = a * x[i] + b;
}

// One "step": three kernels on the capture stream and a forked side stream joined back (the
// shape of the train step's capture: current stream + weight-gradient side stream).
static void step(hipStream_t main, hipStream_t side, hipEvent_t fork, hipEvent_t join, float* a,
                 float* b, float* c, int n) {
  dim3 g((n + 255) / 256), blk(256);
  hipLaunchKernelGGL(axpb, g, blk, 0, main, b, a, 1.5f, 1.0f, n);
  CK(hipEventRecord(fork, main));
  CK(hipStreamWaitEvent(side, fork, 0));
  hipLaunchKernelGGL(axpb, g, blk, 0, side, c, b, 0.5f, -1.0f, n);
  CK(hipEventRecord(join, side));
  hipLaunchKernelGGL(axpb, g, blk, 0, main, a, b, 0.25f, 2.0f, n);
  CK(hipStreamWaitEvent(main, join, 0));
  hipLaunchKernelGGL(axpb, g, blk, 0, main, a, c, 1.0f, 0.0f, n);
}

static int g_reps = 1;

static hipGraphExec_t capture(hipStream_t main, hipStream_t side, float* a, float* b, float* c,
                              int n) {
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  hipGraph_t g;
  CK(hipStreamBeginCapture(main, hipStreamCaptureModeGlobal));
  for (int r = 0; r < g_reps; ++r) step(main, side, fork, join, a, b, c, n);
  CK(hipStreamEndCapture(main, &g));
  hipGraphExec_t x;
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  CK(hipGraphDestroy(g));
  CK(hipEventDestroy(fork));
  CK(hipEventDestroy(join));
  return x;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "two";
  const bool two = strncmp(mode, "two", 3) == 0;
  const bool keep = strstr(mode, "keep") != nullptr;
  const bool big = strstr(mode, "big") != nullptr;
  if (big) g_reps = 64;
  CK(hipSetDevice(0));
  const int n = 1 << 22;
  float *a, *b, *c, *x;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  CK(hipMalloc(&c, n * 4));
  CK(hipMalloc(&x, (1 << 20) * 4));
  CK(hipMemset(a, 0, n * 4));
  CK(hipMemset(x, 0, (1 << 20) * 4));
  hipStream_t main_s, side_s, s2;
  CK(hipStreamCreate(&main_s));
  CK(hipStreamCreate(&side_s));
  CK(hipStreamCreate(&s2));

  // 1. a captured step, replayed (test_graph_steps_vs_oracle)
  hipGraphExec_t g0 = capture(main_s, side_s, a, b, c, n);
  hipStream_t launch_s = big ? (hipStream_t)0 : main_s;
  for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(g0, launch_s));
  CK(hipDeviceSynchronize());
  printf("[%s] graph 0 replayed\n", mode);
  fflush(stdout);

  // 2. a one-rank communicator: all-reduce on the null stream, then (two) on a second stream
  ncclUniqueId id;
  NK(ncclGetUniqueId(&id));
  ncclComm_t comm;
  NK(ncclCommInitRank(&comm, 1, id, 0));
  NK(ncclAllReduce(x, x, 1 << 20, ncclFloat32, ncclSum, comm, 0));
  if (two) {
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipEventRecord(e, 0));
    CK(hipStreamWaitEvent(s2, e, 0));
    NK(ncclAllReduce(x, x, 12345, ncclFloat32, ncclSum, comm, s2));
    CK(hipEventRecord(e, s2));
    CK(hipStreamWaitEvent(0, e, 0));
    CK(hipEventDestroy(e));
  }
  CK(hipDeviceSynchronize());
  if (!keep) NK(ncclCommDestroy(comm));
  printf("[%s] communicator used on %d stream(s), %s\n", mode, two ? 2 : 1,
         keep ? "kept" : "destroyed");
  fflush(stdout);

  // 3. two more captures, each replayed (test_graph_matches_eager, both cases)
  for (int k = 1; k <= 2; ++k) {
    hipGraphExec_t g = capture(main_s, side_s, a, b, c, n);
    for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(g, launch_s));
    CK(hipDeviceSynchronize());
    CK(hipGraphExecDestroy(g));
    printf("[%s] graph %d replayed\n", mode, k);
    fflush(stdout);
  }
  CK(hipGraphExecDestroy(g0));
  if (keep) NK(ncclCommDestroy(comm));
  printf("[%s] ok\n", mode);
  return 0;
}
