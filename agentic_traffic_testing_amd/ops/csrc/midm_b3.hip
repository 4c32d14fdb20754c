// Mid-M GEMM kernels for 48-row blocks (BMT = 3): see midm.h.
#include "midm.h"

namespace atta {
namespace midm {
ATTA_MIDM_TU(3)
}  // namespace midm
}  // namespace atta
