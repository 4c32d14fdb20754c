// Mid-M GEMM kernels for 96-row blocks (BMT = 6): see midm.h.
#include "midm.h"

namespace atta {
namespace midm {
ATTA_MIDM_TU(6)
}  // namespace midm
}  // namespace atta
