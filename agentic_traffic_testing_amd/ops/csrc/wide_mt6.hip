// Wide small-M GEMM kernels for 96-row blocks (MT = 6): see wide.h.
#include "wide.h"

namespace atta {
namespace wide {
ATTA_WIDE_MT_TU(6)
}  // namespace wide
}  // namespace atta
