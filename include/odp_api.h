/*
 * odp_api.h -- umbrella header of the MI355X ODP build (the reference's
 * include/odp_api.h): the runtime subset (odp_rt.h) plus the classification
 * API (odp_cls_api.h).  Applications such as example/classifier include this
 * and link libodp_cls.so (+ libodph.so for the helper).
 */
#ifndef ODP_AMD_API_H_
#define ODP_AMD_API_H_

#include "odp_rt.h"
#include "odp_cls_api.h"

#endif /* ODP_AMD_API_H_ */
