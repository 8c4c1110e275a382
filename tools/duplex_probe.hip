// PCIe duplex probe: do a device->host stream and a host->device stream on different HIP streams
// run at the same time on MI355X (the pipelined host path overlaps the D2H of range r with the
// H2D of range r + 1)?  Pinned buffers, 4 MiB H2D chunks alternating over two streams (the
// session's staging shape) and 16 MiB D2H chunks on a third, alone and together.
// Build: hipcc --offload-arch=gfx950 -O2 tools/duplex_probe.hip -o tools/_duplex_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t h2d_total = 800ull << 20, d2h_total = 400ull << 20;
  const size_t hc = 4ull << 20, dc = 16ull << 20;
  char *hin, *hout, *din, *dout;
  CK(hipHostMalloc((void**)&hin, h2d_total, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&hout, d2h_total, hipHostMallocDefault));
  CK(hipMalloc((void**)&din, h2d_total));
  CK(hipMalloc((void**)&dout, d2h_total));
  for (size_t i = 0; i < h2d_total; i += 4096) hin[i] = (char)i;
  CK(hipMemset(dout, 1, d2h_total));
  hipStream_t s0, s1, s2;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  auto h2d = [&] {
    for (size_t o = 0, i = 0; o < h2d_total; o += hc, ++i)
      CK(hipMemcpyAsync(din + o, hin + o, hc, hipMemcpyHostToDevice, (i & 1) ? s1 : s0));
  };
  auto d2h = [&] {
    for (size_t o = 0; o < d2h_total; o += dc) CK(hipMemcpyAsync(hout + o, dout + o, dc, hipMemcpyDeviceToHost, s2));
  };
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipDeviceSynchronize());
    double t = now();
    h2d();
    CK(hipDeviceSynchronize());
    const double th = now() - t;
    t = now();
    d2h();
    CK(hipDeviceSynchronize());
    const double td = now() - t;
    t = now();
    std::thread a(h2d), b(d2h);
    a.join();
    b.join();
    CK(hipDeviceSynchronize());
    const double tb = now() - t;
    printf("{\"rep\": %d, \"h2d_ms\": %.2f, \"h2d_GBps\": %.1f, \"d2h_ms\": %.2f, \"d2h_GBps\": %.1f, "
           "\"both_ms\": %.2f, \"sum_ms\": %.2f, \"overlap\": %.2f}\n",
           rep, th * 1e3, h2d_total / th / 1e9, td * 1e3, d2h_total / td / 1e9, tb * 1e3, (th + td) * 1e3,
           (th + td - tb) / std::min(th, td));
    fflush(stdout);
  }
  return 0;
}
