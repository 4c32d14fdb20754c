// Wide small-M GEMM kernels for 16-row blocks (MT = 1): see wide.h.
#include "wide.h"

namespace atta {
namespace wide {
ATTA_WIDE_MT_TU(1)
}  // namespace wide
}  // namespace atta
