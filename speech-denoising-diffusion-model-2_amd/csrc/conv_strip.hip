// Row-streaming 3x3 convolution: host entry points (kernel in conv_strip_impl.h, instantiated per
// storage type in conv_strip_{bf16,f16,f32}.hip).
#include "kernels.h"
#include "sddm_common.h"

namespace sddm {

template <typename T>
hipError_t strip_dispatch(const ConvArgs& a, int nblk, int mpi, int SR, int B, hipStream_t s, size_t* lo);
extern template hipError_t strip_dispatch<bf16_t>(const ConvArgs&, int, int, int, int, hipStream_t, size_t*);
extern template hipError_t strip_dispatch<f16_t>(const ConvArgs&, int, int, int, int, hipStream_t, size_t*);
extern template hipError_t strip_dispatch<float>(const ConvArgs&, int, int, int, int, hipStream_t, size_t*);

hipError_t launch_conv_strip(int dtype, int nblk, int mpi, int SR, const ConvArgs& a, int B, hipStream_t s) {
  if (dtype == DT_F32) return strip_dispatch<float>(a, nblk, mpi, SR, B, s, nullptr);
  if (dtype == DT_BF16) return strip_dispatch<bf16_t>(a, nblk, mpi, SR, B, s, nullptr);
  return strip_dispatch<f16_t>(a, nblk, mpi, SR, B, s, nullptr);
}

size_t conv_strip_lds_bytes(int dtype, int nblk, int mpi, const ConvArgs& a) {
  size_t lo = (size_t)1 << 40;
  if (dtype == DT_F32) (void)strip_dispatch<float>(a, nblk, mpi, 1, 1, 0, &lo);
  else if (dtype == DT_BF16) (void)strip_dispatch<bf16_t>(a, nblk, mpi, 1, 1, 0, &lo);
  else (void)strip_dispatch<f16_t>(a, nblk, mpi, 1, 1, 0, &lo);
  return lo;
}

}  // namespace sddm
