// mi_cls_ks.hip -- A/B builds only: a program-specialised flat kernel
// (4-wave blocks) whose block comes from a spec file dumped by
// MI_CLS_DUMP_SPEC (odp_amd/_build.py: MI_SPEC_FILE="..."); launched when
// MI_CLS_SPEC_LAUNCH is set.  Product builds compile the stub.
#include "mi_cls_dev.h"

#ifdef MI_SPEC_FILE
#include MI_SPEC_FILE
int mi_cls_launch_spec(unsigned grid, size_t dyn, hipStream_t st, const KArgs &a)
{
	hipLaunchKernelGGL((mi_cls_kernel<true, false, 4, MI_SPEC_FM, false, MiSpec>), dim3(grid),
			   dim3(4 * WAVE), dyn, st, a);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
#else
int mi_cls_launch_spec(unsigned, size_t, hipStream_t, const KArgs &)
{
	return -ENOSYS;
}
#endif
