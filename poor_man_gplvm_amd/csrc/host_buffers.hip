// Page-locked host buffers for the arrays a fit returns (core.run_em: posterior, log
// posterior, marginals; core.py:696-712 in the reference returns them as host arrays).
//
// A fresh page-locked allocation costs mostly the kernel's zero-fill of each new page on
// first touch (≈34 ms for 410 MB through torch's pinned allocator, one thread).  Here the
// pages are mapped anonymously, first-touched by `threads` host threads in parallel
// (optionally as transparent huge pages), and only then registered with HIP, so the pin
// itself walks already-present pages.  The caller may run this on a side thread while the
// device computes: the C call holds no Python lock.
#include <sys/mman.h>

#include <thread>
#include <vector>

#include "pmg_common.h"

namespace {
constexpr size_t kPage = 4096;
}

extern "C" int pmg_host_alloc(size_t bytes, int32_t threads, int32_t huge, void** out) {
  PMG_REQUIRE(out != nullptr && bytes > 0, "pmg_host_alloc: null output or zero size");
  *out = nullptr;
  const size_t len = (bytes + kPage - 1) / kPage * kPage;
  void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  PMG_REQUIRE(p != MAP_FAILED, "pmg_host_alloc: mmap of %zu bytes failed", len);
  if (huge) madvise(p, len, MADV_HUGEPAGE);
  const int nt = threads < 1 ? 1 : (threads > 64 ? 64 : threads);
  const size_t pages = len / kPage;
  auto touch = [p](size_t a, size_t b) {
    volatile char* c = static_cast<char*>(p);
    for (size_t i = a; i < b; ++i) c[i * kPage] = 0;
  };
  if (nt == 1 || pages < 1024) {
    touch(0, pages);
  } else {
    std::vector<std::thread> ts;
    const size_t per = (pages + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
      const size_t a = t * per, b = a + per < pages ? a + per : pages;
      if (a < b) ts.emplace_back(touch, a, b);
    }
    for (auto& t : ts) t.join();
  }
  const hipError_t e = hipHostRegister(p, len, hipHostRegisterDefault);
  if (e != hipSuccess) {
    munmap(p, len);
    ::pmg::set_error("pmg_host_alloc: hipHostRegister(%zu bytes): %s", len, hipGetErrorString(e));
    return PMG_EHIP;
  }
  *out = p;
  return PMG_OK;
}

extern "C" int pmg_host_free(void* p, size_t bytes) {
  if (p == nullptr) return PMG_OK;
  const size_t len = (bytes + kPage - 1) / kPage * kPage;
  const hipError_t e = hipHostUnregister(p);
  munmap(p, len);
  PMG_REQUIRE(e == hipSuccess, "pmg_host_free: hipHostUnregister: %s", hipGetErrorString(e));
  return PMG_OK;
}

// device -> host copy of `bytes` into a pmg_host_alloc buffer, enqueued on `stream`
// (the caller synchronises the stream before reading dst)
extern "C" int pmg_copy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
  if (bytes == 0) return PMG_OK;   // nothing to copy (an empty tensor's data pointer is NULL)
  PMG_REQUIRE(dst != nullptr && src != nullptr, "pmg_copy_d2h: null pointer");
  PMG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ::pmg::as_stream(stream)));
  return PMG_OK;
}
