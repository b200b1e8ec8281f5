// mi_cls_kc16.hip -- pktin-option instantiations of mi_cls_kernel (CK) for
// the 16-wave, one-block-per-CU shape with the hot region in LDS (see
// mi_cls_kc4.hip).
#include "mi_cls_dev.h"

int mi_cls_launch_ck16(bool div, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a)
{
	if (div)
		MI_LAUNCH((mi_cls_kernel<true, true, 16, -1, true>), grid, 16 * WAVE, dyn, st, a);
	else
		MI_LAUNCH((mi_cls_kernel<true, false, 16, -1, true>), grid, 16 * WAVE, dyn, st, a);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
