// Mid-M GEMM kernels for 160-row blocks (BMT = 10): see midm.h.
#include "midm.h"

namespace atta {
namespace midm {
ATTA_MIDM_TU(10)
}  // namespace midm
}  // namespace atta
