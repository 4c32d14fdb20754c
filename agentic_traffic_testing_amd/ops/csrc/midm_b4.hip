// Mid-M GEMM kernels for 64-row blocks (BMT = 4): see midm.h.
#include "midm.h"

namespace atta {
namespace midm {
ATTA_MIDM_TU(4)
}  // namespace midm
}  // namespace atta
