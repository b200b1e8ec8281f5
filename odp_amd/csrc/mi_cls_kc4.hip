// mi_cls_kc4.hip -- pktin-option instantiations of mi_cls_kernel (CK: IPv4 /
// L4 checksum validation and drop-on-error options, odp_pktio_config()
// pktin bits) for the 4-wave block shape.  A program with pktin options runs
// these (4-wave blocks, or mi_cls_kc16.hip's 16-wave blocks when the hot
// region needs the shared LDS copy); the option-free kernels carry none of
// this code.
#include "mi_cls_dev.h"

int mi_cls_launch_ck16(bool div, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a);

int mi_cls_launch_ck(int nw, bool lt, bool div, unsigned grid, size_t dyn, hipStream_t st,
		     const KArgs &a)
{
	if (nw == 16 && lt)
		return mi_cls_launch_ck16(div, grid, dyn, st, a);
	if (nw != 4)
		return -EINVAL;
	if (lt && div)
		MI_LAUNCH((mi_cls_kernel<true, true, 4, -1, true>), grid, 4 * WAVE, dyn, st, a);
	else if (lt)
		MI_LAUNCH((mi_cls_kernel<true, false, 4, -1, true>), grid, 4 * WAVE, dyn, st, a);
	else if (div)
		MI_LAUNCH((mi_cls_kernel<false, true, 4, -1, true>), grid, 4 * WAVE, dyn, st, a);
	else
		MI_LAUNCH((mi_cls_kernel<false, false, 4, -1, true>), grid, 4 * WAVE, dyn, st, a);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
