// conv_strip_kernel instantiations for bf16_t storage (conv_strip_impl.h; one translation unit per
// storage type so the three compile in parallel)
#include "conv_strip_impl.h"

namespace sddm {
template hipError_t strip_dispatch<bf16_t>(const ConvArgs&, int, int, int, int, hipStream_t, size_t*);
}  // namespace sddm
