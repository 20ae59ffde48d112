// graph_overhead.hip -- host-side cost of the chain's hipGraph launch path on this ROCm, measured
// on 5 dependent tiny kernels (the chain's FEC x 3, map, OFDM node count):
//   direct   : 5 hipLaunchKernelGGL + hipStreamSynchronize
//   graph    : hipGraphLaunch of the captured chain + sync (no argument update)
//   setparams: 5 hipGraphExecKernelNodeSetParams + hipGraphLaunch + sync
//   enqueue  : host time of the calls alone (no sync), per variant
// Prints one JSON line.  Experiment tooling, not product.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

struct Args {
  int *p;
  int a, b, c, d;
  long long e;
};

__global__ void tiny(Args x) {
  if (threadIdx.x == 0 && blockIdx.x == 0) x.p[0] += x.a + x.b;
}

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  int *p;
  CK(hipMalloc(&p, 64));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int NK = 5, REP = 200;
  Args a{p, 1, 2, 3, 4, 5};
  auto launch5 = [&](hipStream_t st) {
    for (int k = 0; k < NK; k++) hipLaunchKernelGGL(tiny, dim3(64), dim3(256), 0, st, a);
  };
  // capture
  hipStream_t cs;
  CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  hipGraph_t g;
  CK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
  launch5(cs);
  CK(hipStreamEndCapture(cs, &g));
  hipGraphExec_t ex;
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  size_t n = 0;
  CK(hipGraphGetNodes(g, nullptr, &n));
  std::vector<hipGraphNode_t> nodes(n);
  CK(hipGraphGetNodes(g, nodes.data(), &n));
  std::vector<hipKernelNodeParams> base(n);
  for (size_t i = 0; i < n; i++) CK(hipGraphKernelNodeGetParams(nodes[i], &base[i]));
  std::vector<double> t_direct, t_graph, t_set, e_direct, e_graph, e_set;
  for (int r = 0; r < REP; r++) {
    a.a = r;
    double t0 = now_us();
    launch5(s);
    double t1 = now_us();
    CK(hipStreamSynchronize(s));
    double t2 = now_us();
    t_direct.push_back(t2 - t0);
    e_direct.push_back(t1 - t0);
    t0 = now_us();
    CK(hipGraphLaunch(ex, s));
    t1 = now_us();
    CK(hipStreamSynchronize(s));
    t2 = now_us();
    t_graph.push_back(t2 - t0);
    e_graph.push_back(t1 - t0);
    t0 = now_us();
    void *args[1] = {&a};
    for (size_t i = 0; i < n; i++) {
      hipKernelNodeParams kp = base[i];
      kp.kernelParams = args;
      kp.extra = nullptr;
      CK(hipGraphExecKernelNodeSetParams(ex, nodes[i], &kp));
    }
    CK(hipGraphLaunch(ex, s));
    t1 = now_us();
    CK(hipStreamSynchronize(s));
    t2 = now_us();
    t_set.push_back(t2 - t0);
    e_set.push_back(t1 - t0);
  }
  auto med = [](std::vector<double> v) {
    v.erase(v.begin(), v.begin() + 20);
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  std::printf("{\"nodes\": %zu, \"direct_us\": %.2f, \"direct_enqueue_us\": %.2f, \"graph_us\": %.2f, "
              "\"graph_enqueue_us\": %.2f, \"setparams_graph_us\": %.2f, \"setparams_graph_enqueue_us\": %.2f}\n",
              n, med(t_direct), med(e_direct), med(t_graph), med(e_graph), med(t_set), med(e_set));
  return 0;
}
