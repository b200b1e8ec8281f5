// mi_cls_k4.hip -- the 4-wave block shape of mi_cls_kernel (one
// translation unit per shape so the shapes compile in parallel).
#include "mi_cls_dev.h"

int mi_cls_launch_k4(bool lt, bool div, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a)
{
	if (lt && div)
		MI_LAUNCH((mi_cls_kernel<true, true, 4>), grid, 4 * WAVE, dyn, st, a);
	else if (lt)
		MI_LAUNCH((mi_cls_kernel<true, false, 4>), grid, 4 * WAVE, dyn, st, a);
	else if (div)
		MI_LAUNCH((mi_cls_kernel<false, true, 4>), grid, 4 * WAVE, dyn, st, a);
	else
		MI_LAUNCH((mi_cls_kernel<false, false, 4>), grid, 4 * WAVE, dyn, st, a);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
