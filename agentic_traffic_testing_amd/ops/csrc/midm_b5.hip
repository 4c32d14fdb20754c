// Mid-M GEMM kernels for 80-row blocks (BMT = 5): see midm.h.
#include "midm.h"

namespace atta {
namespace midm {
ATTA_MIDM_TU(5)
}  // namespace midm
}  // namespace atta
