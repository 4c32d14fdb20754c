// Mid-M GEMM kernels for 128-row blocks (BMT = 8): see midm.h.
#include "midm.h"

namespace atta {
namespace midm {
ATTA_MIDM_TU(8)
}  // namespace midm
}  // namespace atta
