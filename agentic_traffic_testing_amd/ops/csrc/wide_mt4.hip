// Wide small-M GEMM kernels for 64-row blocks (MT = 4): see wide.h.
#include "wide.h"

namespace atta {
namespace wide {
ATTA_WIDE_MT_TU(4)
}  // namespace wide
}  // namespace atta
