// TEST INFRASTRUCTURE ONLY -- the LDS backing store of the SIMT emulation,
// for build/so/libsimt_lzma.so: the product C ABI (lzma-java_amd/csrc)
// compiled for the CPU emulation as a shared library, so multi-process CPU
// tests (gloo) can run the product kernels' logic without a GPU.
#include <stdint.h>
namespace lzg { alignas(16) uint8_t smem[160 * 1024]; namespace sliced { alignas(16) uint8_t smem[160 * 1024]; } }
