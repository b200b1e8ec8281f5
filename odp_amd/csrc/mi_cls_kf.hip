// mi_cls_kf.hip -- flat-program instantiations of mi_cls_kernel: the default
// CoS decides every packet in one round with a compile-time engine (direct,
// bitmap, wide bitmap, single candidate), hot region in LDS, no pktin
// options.  One translation unit per block shape (mi_cls_kf.hip: 4 waves and
// the dispatcher, mi_cls_kf12.hip, mi_cls_kf16.hip) so they compile in
// parallel beside the general shapes.
#include "mi_cls_dev.h"

int mi_cls_launch_flat12(int fm, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a);
int mi_cls_launch_flat16(int fm, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a);

template <int NW>
static int launch_fm(int fm, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a)
{
	switch (fm) {
	case 0:
		MI_LAUNCH((mi_cls_kernel<true, false, NW, 0>), grid, NW * WAVE, dyn, st, a);
		break;
	case 2:
		MI_LAUNCH((mi_cls_kernel<true, false, NW, 2>), grid, NW * WAVE, dyn, st, a);
		break;
	case 3:
		MI_LAUNCH((mi_cls_kernel<true, false, NW, 3>), grid, NW * WAVE, dyn, st, a);
		break;
	case 4:
		MI_LAUNCH((mi_cls_kernel<true, false, NW, 4>), grid, NW * WAVE, dyn, st, a);
		break;
	default:
		return -EINVAL;
	}
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

int mi_cls_launch_flat(int nw, int fm, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a)
{
	if (nw == 16)
		return mi_cls_launch_flat16(fm, grid, dyn, st, a);
	if (nw == 12)
		return mi_cls_launch_flat12(fm, grid, dyn, st, a);
	if (nw == 4)
		return launch_fm<4>(fm, grid, dyn, st, a);
	return -EINVAL;
}
