// Host->device copy rate from pinned memory: chunk size x number of HIP streams the chunks are
// spread over (does a second DMA queue raise the H2D rate the session's staging ring gets?).
// Build: hipcc --offload-arch=gfx950 -O2 tools/h2d_probe.hip -o tools/_h2d_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

int main() {
  const size_t total = 1ull << 30;  // 1 GiB per measurement
  char* h = nullptr;
  char* d = nullptr;
  CK(hipHostMalloc((void**)&h, total, hipHostMallocDefault));
  CK(hipMalloc((void**)&d, total));
  for (size_t i = 0; i < total; i += 4096) h[i] = (char)i;
  std::vector<hipStream_t> st(4);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t chunks[] = {1ull << 20, 4ull << 20, 16ull << 20, 64ull << 20};
  for (int dir = 0; dir < 2; ++dir) {
    for (size_t cb : chunks) {
      for (int ns : {1, 2, 4}) {
        double best = 0;
        for (int rep = 0; rep < 5; ++rep) {
          CK(hipDeviceSynchronize());
          auto t0 = std::chrono::steady_clock::now();
          for (size_t off = 0, u = 0; off < total; off += cb, ++u) {
            hipStream_t s = st[u % ns];
            if (dir == 0)
              CK(hipMemcpyAsync(d + off, h + off, cb, hipMemcpyHostToDevice, s));
            else
              CK(hipMemcpyAsync(h + off, d + off, cb, hipMemcpyDeviceToHost, s));
          }
          for (int i = 0; i < ns; ++i) CK(hipStreamSynchronize(st[i]));
          double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
          if (rep > 0 && total / sec / 1e9 > best) best = total / sec / 1e9;
        }
        printf("{\"dir\": \"%s\", \"chunk_MiB\": %zu, \"streams\": %d, \"GBps\": %.1f}\n", dir ? "d2h" : "h2d",
               cb >> 20, ns, best);
        fflush(stdout);
      }
    }
  }
  return 0;
}
