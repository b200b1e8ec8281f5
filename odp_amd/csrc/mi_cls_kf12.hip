// mi_cls_kf12.hip -- flat-program instantiations of mi_cls_kernel for the
// 12-wave block shape (see mi_cls_kf.hip).
#include "mi_cls_dev.h"

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

int mi_cls_launch_flat12(int fm, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a)
{
	return launch_fm<12>(fm, grid, dyn, st, a);
}
