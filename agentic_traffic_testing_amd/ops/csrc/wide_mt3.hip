// Wide small-M GEMM kernels for 48-row blocks (MT = 3): see wide.h.
#include "wide.h"

namespace atta {
namespace wide {
ATTA_WIDE_MT_TU(3)
}  // namespace wide
}  // namespace atta
