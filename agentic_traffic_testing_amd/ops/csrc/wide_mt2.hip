// Wide small-M GEMM kernels for 32-row blocks (MT = 2): see wide.h.
#include "wide.h"

namespace atta {
namespace wide {
ATTA_WIDE_MT_TU(2)
}  // namespace wide
}  // namespace atta
