#include "bsg_kernels.hip"
namespace bsg {
template <int KIND, int GS>
__global__ __launch_bounds__(64) void la_only_kernel(KParams p) {
  __shared__ Lds<false> L;
  constexpr int kList = 64 * (GS > 1 ? GS - 1 : 1);
  __shared__ unsigned short cd_lists[kList];
  lookahead_role<KIND, GS, false, 1>(p, L, cd_lists);
}
template __global__ void la_only_kernel<BSG_ENV_MERGE, 32>(KParams);
}
