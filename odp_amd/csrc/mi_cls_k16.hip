// mi_cls_k16.hip -- the 16-wave block shape of mi_cls_kernel (one
// translation unit per shape so the shapes compile in parallel).
#include "mi_cls_dev.h"

int mi_cls_launch_k16(bool lt, bool div, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a)
{
	if (lt && div)
		MI_LAUNCH((mi_cls_kernel<true, true, 16>), grid, 16 * WAVE, dyn, st, a);
	else if (lt)
		MI_LAUNCH((mi_cls_kernel<true, false, 16>), grid, 16 * WAVE, dyn, st, a);
	else if (div)
		MI_LAUNCH((mi_cls_kernel<false, true, 16>), grid, 16 * WAVE, dyn, st, a);
	else
		MI_LAUNCH((mi_cls_kernel<false, false, 16>), grid, 16 * WAVE, dyn, st, a);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
