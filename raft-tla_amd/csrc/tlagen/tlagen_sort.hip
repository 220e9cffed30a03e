// tlagen_sort.hip — the one library kernel the generated path needs that is not generated: the
// radix sort of a level's winner keys in TLC's FIFO order (tlagen_kernels.h, pass 1 -> pass 2).
// The generated code object (hiprtc) holds the spec's kernels; the sort is spec independent.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

namespace rmc {

// keys_in[0, n) -> keys_out ascending over the low `bits` bits; *tmp / *tmp_bytes grow as needed
int tlagen_sort_keys(const unsigned long long* keys_in, unsigned long long* keys_out, unsigned long long n, int bits,
                     void** tmp, size_t* tmp_bytes, hipStream_t s) {
  size_t need = 0;
  if (rocprim::radix_sort_keys(nullptr, need, keys_in, keys_out, (size_t)n, 0, bits, s) != hipSuccess) return -1;
  if (need > *tmp_bytes) {
    if (*tmp) (void)hipFree(*tmp);
    *tmp = nullptr;
    *tmp_bytes = 0;
    if (hipMalloc(tmp, need) != hipSuccess) return -2;
    *tmp_bytes = need;
  }
  size_t have = *tmp_bytes;
  if (rocprim::radix_sort_keys(*tmp, have, keys_in, keys_out, (size_t)n, 0, bits, s) != hipSuccess) return -1;
  return 0;
}

}  // namespace rmc
