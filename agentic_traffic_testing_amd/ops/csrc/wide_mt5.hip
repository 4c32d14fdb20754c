// Wide small-M GEMM kernels for 80-row blocks (MT = 5): see wide.h.
#include "wide.h"

namespace atta {
namespace wide {
ATTA_WIDE_MT_TU(5)
}  // namespace wide
}  // namespace atta
