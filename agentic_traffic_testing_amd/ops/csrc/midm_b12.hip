// Mid-M GEMM kernels for 192-row blocks (BMT = 12): see midm.h.
#include "midm.h"

namespace atta {
namespace midm {
ATTA_MIDM_TU(12)
}  // namespace midm
}  // namespace atta
