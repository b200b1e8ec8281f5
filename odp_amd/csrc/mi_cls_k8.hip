// mi_cls_k8.hip -- the 8-wave block shape of mi_cls_kernel (one
// translation unit per shape so the shapes compile in parallel).
#include "mi_cls_dev.h"

int mi_cls_launch_k8(bool lt, bool div, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a)
{
	(void)lt;   // 8-wave blocks exist for LDS-resident hot regions only
	if (div)
		MI_LAUNCH((mi_cls_kernel<true, true, 8>), grid, 8 * WAVE, dyn, st, a);
	else
		MI_LAUNCH((mi_cls_kernel<true, false, 8>), grid, 8 * WAVE, dyn, st, a);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
