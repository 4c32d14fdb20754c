// Wide small-M GEMM kernels for 112-row blocks (MT = 7): see wide.h.
#include "wide.h"

namespace atta {
namespace wide {
ATTA_WIDE_MT_TU(7)
}  // namespace wide
}  // namespace atta
