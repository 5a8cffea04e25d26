// launch_cost.hip — host cost of one kernel launch by API (bb_plan_launch's replay choice) and
// the event-bracketed latency of two dependent 1-workgroup launches, as request_latency sees
// a search: hipLaunchKernelGGL, hipLaunchKernel(stub, argv), hipModuleLaunchKernel(func from
// hipGetFuncBySymbol, argv), hipModuleLaunchKernel(func, extra = packed argument buffer).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/launch_cost.hip -o tools/launch_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>
#include <functional>

struct Big {  // a SqArgs-sized kernel argument
  float* out;
  int v[124];
};

__global__ void k_big(Big a) {
  if (threadIdx.x == 0 && blockIdx.x == 0) a.out[0] = (float)a.v[3];
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  float* out;
  (void)hipMalloc(&out, 4096);
  Big b{};
  b.out = out;
  for (int i = 0; i < 124; ++i) b.v[i] = i;
  void* argv[1] = {&b};
  hipFunction_t f = nullptr;
  hipError_t e = hipGetFuncBySymbol(&f, (const void*)k_big);
  printf("{\"hipGetFuncBySymbol\": %d}\n", (int)e);
  size_t sz = sizeof(Big);
  void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &b, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  auto ggl = [&] { hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, b); };
  auto stub = [&] { (void)hipLaunchKernel((const void*)k_big, dim3(1), dim3(64), argv, 0, s); };
  auto mod = [&] { (void)hipModuleLaunchKernel(f, 1, 1, 1, 64, 1, 1, 0, s, argv, nullptr); };
  auto modx = [&] { (void)hipModuleLaunchKernel(f, 1, 1, 1, 64, 1, 1, 0, s, nullptr, extra); };
  struct V { const char* name; std::function<void()> fn; };
  std::vector<std::pair<const char*, std::function<void()>>> vs = {
      {"hipLaunchKernelGGL", ggl}, {"hipLaunchKernel", stub}, {"hipModuleLaunchKernel_argv", mod},
      {"hipModuleLaunchKernel_extra", modx}};
  hipEvent_t a, z;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&z);
  for (auto& [name, fn] : vs) {
    if (!f && std::strstr(name, "Module")) continue;
    for (int i = 0; i < 100; ++i) fn();
    (void)hipStreamSynchronize(s);
    // host cost per launch (queue never full: sync every 32)
    std::vector<double> host;
    for (int r = 0; r < 64; ++r) {
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < 16; ++i) fn();
      auto t1 = std::chrono::steady_clock::now();
      host.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / 16);
      (void)hipStreamSynchronize(s);
    }
    // serial: event, two dependent launches, event (idle stream each time)
    std::vector<double> ser, single;
    for (int r = 0; r < 200; ++r) {
      (void)hipEventRecord(a, s);
      fn();
      fn();
      (void)hipEventRecord(z, s);
      (void)hipEventSynchronize(z);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, z);
      ser.push_back(ms * 1e3);
      (void)hipEventRecord(a, s);
      fn();
      (void)hipEventRecord(z, s);
      (void)hipEventSynchronize(z);
      (void)hipEventElapsedTime(&ms, a, z);
      single.push_back(ms * 1e3);
    }
    std::sort(host.begin(), host.end());
    std::sort(ser.begin(), ser.end());
    std::sort(single.begin(), single.end());
    float chk = 0;
    (void)hipMemcpy(&chk, out, 4, hipMemcpyDeviceToHost);
    printf("{\"api\":\"%s\",\"host_us_per_launch_p50\":%.3f,\"event_us_two_launches_p50\":%.2f,"
           "\"event_us_one_launch_p50\":%.2f,\"check\":%.0f}\n",
           name, host[host.size() / 2], ser[ser.size() / 2], single[single.size() / 2], chk);
  }
  return 0;
}
