// Wide small-M GEMM kernels for 128-row blocks (MT = 8): see wide.h.
#include "wide.h"

namespace atta {
namespace wide {
ATTA_WIDE_MT_TU(8)
}  // namespace wide
}  // namespace atta
