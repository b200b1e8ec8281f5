/*
 * odp_rt.h -- the ODP runtime subset served by the MI355X build: the types and
 * calls an ODP application around the classifier receive path uses
 * (init, shm, pools, packets, events, queues, scheduler, packet I/O, time,
 * cpumask, threads, atomics, byte order).  SURVEY.md Appendix C lists what
 * example/classifier/odp_classifier.c consumes; this header supplies those
 * names with the reference's field paths, enum values and error returns so
 * that file compiles unchanged.
 *
 * Spec files followed (include/odp/api/spec/): init.h, shared_memory.h,
 * pool.h + pool_types.h, packet.h + packet_flags.h, event.h,
 * event_vector.h + event_vector_types.h, queue.h + queue_types.h,
 * schedule.h + schedule_types.h, packet_io.h + packet_io_types.h +
 * packet_io_stats.h, time.h, cpumask.h, thread.h, atomic.h, spinlock.h,
 * byteorder.h, system_info.h; ABI constants from include/odp/api/abi-default/.
 *
 * Handles are opaque pointers; every *_INVALID is 0.  What is not part of
 * the receive path is deliberately small (pools, queues and
 * schedulers only as far as §8(f) rank 1 needs them).
 */
#ifndef ODP_AMD_RT_H_
#define ODP_AMD_RT_H_

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------ basics */
typedef bool odp_bool_t;

#define odp_likely(x)   __builtin_expect(!!(x), 1)
#define odp_unlikely(x) __builtin_expect(!!(x), 0)
#define ODP_UNUSED      __attribute__((__unused__))
#define ODP_ALIGNED(x)  __attribute__((__aligned__(x)))
#define ODP_ALIGNED_CACHE ODP_ALIGNED(ODP_CACHE_LINE_SIZE)
#define ODP_PRINTF_FORMAT(a, b) __attribute__((format(printf, a, b)))
#define ODP_STATIC_ASSERT(cond, msg) _Static_assert(cond, msg)
#define ODP_CACHE_LINE_SIZE 64
#define ODP_PAGE_SIZE 4096

typedef enum { ODP_SUPPORT_NO = 0, ODP_SUPPORT_YES, ODP_SUPPORT_PREFERRED } odp_support_t;

/* opaque pointer-sized handles, 0 == INVALID (abi-default headers) */
typedef struct _odp_abi_cos_t    *odp_cos_t;
typedef struct _odp_abi_pmr_t    *odp_pmr_t;
typedef struct _odp_abi_queue_t  *odp_queue_t;
typedef struct _odp_abi_pool_t   *odp_pool_t;
typedef struct _odp_abi_pktio_t  *odp_pktio_t;
typedef struct _odp_abi_packet_t *odp_packet_t;
typedef struct _odp_abi_event_t  *odp_event_t;
typedef struct _odp_abi_evv_t    *odp_event_vector_t;
typedef struct _odp_abi_pktv_t   *odp_packet_vector_t;
typedef struct _odp_abi_shm_t    *odp_shm_t;
typedef struct _odp_abi_pktin_t  *_odp_pktin_hdl_t;
typedef uint64_t odp_instance_t;

#define ODP_COS_INVALID    ((odp_cos_t)0)
#define ODP_PMR_INVALID    ((odp_pmr_t)0)
#define ODP_QUEUE_INVALID  ((odp_queue_t)0)
#define ODP_POOL_INVALID   ((odp_pool_t)0)
#define ODP_PKTIO_INVALID  ((odp_pktio_t)0)
#define ODP_PACKET_INVALID ((odp_packet_t)0)
#define ODP_EVENT_INVALID  ((odp_event_t)0)
#define ODP_EVENT_VECTOR_INVALID ((odp_event_vector_t)0)
#define ODP_PACKET_VECTOR_INVALID ((odp_packet_vector_t)0)
#define ODP_SHM_INVALID    ((odp_shm_t)0)

#define ODP_COS_NAME_LEN    32
#define ODP_POOL_NAME_LEN   32
#define ODP_QUEUE_NAME_LEN  32
#define ODP_PKTIO_NAME_LEN  256   /* PKTIO_NAME_LEN, odp_packet_io_internal.h:51 */
#define ODP_SHM_NAME_LEN    32
#define ODP_THREAD_COUNT_MAX 256
#define ODP_PKTIN_MAX_QUEUES  64
#define ODP_PKTOUT_MAX_QUEUES 64
#define ODP_PACKET_OFFSET_INVALID 0xffff

/* ------------------------------------------------------------ byte order */
typedef uint16_t odp_u16be_t;
typedef uint32_t odp_u32be_t;
typedef uint64_t odp_u64be_t;
typedef uint16_t odp_u16sum_t;
typedef uint32_t odp_u32sum_t;

static inline uint16_t odp_cpu_to_be_16(uint16_t v) { return __builtin_bswap16(v); }
static inline uint32_t odp_cpu_to_be_32(uint32_t v) { return __builtin_bswap32(v); }
static inline uint64_t odp_cpu_to_be_64(uint64_t v) { return __builtin_bswap64(v); }
static inline uint16_t odp_be_to_cpu_16(uint16_t v) { return __builtin_bswap16(v); }
static inline uint32_t odp_be_to_cpu_32(uint32_t v) { return __builtin_bswap32(v); }
static inline uint64_t odp_be_to_cpu_64(uint64_t v) { return __builtin_bswap64(v); }

/* ------------------------------------------------------------ atomics */
typedef struct { uint32_t v; } ODP_ALIGNED(4) odp_atomic_u32_t;
typedef struct { uint64_t v; } ODP_ALIGNED(8) odp_atomic_u64_t;

static inline void odp_atomic_init_u32(odp_atomic_u32_t *a, uint32_t v) { __atomic_store_n(&a->v, v, __ATOMIC_RELAXED); }
static inline uint32_t odp_atomic_load_u32(odp_atomic_u32_t *a) { return __atomic_load_n(&a->v, __ATOMIC_RELAXED); }
static inline void odp_atomic_store_u32(odp_atomic_u32_t *a, uint32_t v) { __atomic_store_n(&a->v, v, __ATOMIC_RELAXED); }
static inline void odp_atomic_inc_u32(odp_atomic_u32_t *a) { (void)__atomic_fetch_add(&a->v, 1, __ATOMIC_RELAXED); }
static inline void odp_atomic_dec_u32(odp_atomic_u32_t *a) { (void)__atomic_fetch_sub(&a->v, 1, __ATOMIC_RELAXED); }
static inline void odp_atomic_add_u32(odp_atomic_u32_t *a, uint32_t v) { (void)__atomic_fetch_add(&a->v, v, __ATOMIC_RELAXED); }
static inline void odp_atomic_sub_u32(odp_atomic_u32_t *a, uint32_t v) { (void)__atomic_fetch_sub(&a->v, v, __ATOMIC_RELAXED); }
static inline uint32_t odp_atomic_fetch_inc_u32(odp_atomic_u32_t *a) { return __atomic_fetch_add(&a->v, 1, __ATOMIC_RELAXED); }
static inline uint32_t odp_atomic_fetch_add_u32(odp_atomic_u32_t *a, uint32_t v) { return __atomic_fetch_add(&a->v, v, __ATOMIC_RELAXED); }
static inline void odp_atomic_init_u64(odp_atomic_u64_t *a, uint64_t v) { __atomic_store_n(&a->v, v, __ATOMIC_RELAXED); }
static inline uint64_t odp_atomic_load_u64(odp_atomic_u64_t *a) { return __atomic_load_n(&a->v, __ATOMIC_RELAXED); }
static inline void odp_atomic_store_u64(odp_atomic_u64_t *a, uint64_t v) { __atomic_store_n(&a->v, v, __ATOMIC_RELAXED); }
static inline void odp_atomic_inc_u64(odp_atomic_u64_t *a) { (void)__atomic_fetch_add(&a->v, 1, __ATOMIC_RELAXED); }
static inline void odp_atomic_dec_u64(odp_atomic_u64_t *a) { (void)__atomic_fetch_sub(&a->v, 1, __ATOMIC_RELAXED); }
static inline void odp_atomic_add_u64(odp_atomic_u64_t *a, uint64_t v) { (void)__atomic_fetch_add(&a->v, v, __ATOMIC_RELAXED); }
static inline void odp_atomic_sub_u64(odp_atomic_u64_t *a, uint64_t v) { (void)__atomic_fetch_sub(&a->v, v, __ATOMIC_RELAXED); }
static inline uint64_t odp_atomic_fetch_inc_u64(odp_atomic_u64_t *a) { return __atomic_fetch_add(&a->v, 1, __ATOMIC_RELAXED); }
static inline uint64_t odp_atomic_fetch_add_u64(odp_atomic_u64_t *a, uint64_t v) { return __atomic_fetch_add(&a->v, v, __ATOMIC_RELAXED); }

/* ------------------------------------------------------------ spinlock */
typedef struct { char lock; } odp_spinlock_t;

static inline void odp_spinlock_init(odp_spinlock_t *l) { __atomic_clear(&l->lock, __ATOMIC_RELAXED); }
static inline int odp_spinlock_trylock(odp_spinlock_t *l) { return !__atomic_test_and_set(&l->lock, __ATOMIC_ACQUIRE); }
static inline void odp_spinlock_lock(odp_spinlock_t *l)
{
	while (__atomic_test_and_set(&l->lock, __ATOMIC_ACQUIRE))
		while (__atomic_load_n(&l->lock, __ATOMIC_RELAXED))
			__builtin_ia32_pause();
}
static inline void odp_spinlock_unlock(odp_spinlock_t *l) { __atomic_clear(&l->lock, __ATOMIC_RELEASE); }
static inline int odp_spinlock_is_locked(odp_spinlock_t *l) { return __atomic_load_n(&l->lock, __ATOMIC_RELAXED) != 0; }

/* ------------------------------------------------------------ time */
typedef union {
	uint64_t nsec;
	uint64_t u64;
} odp_time_t;

#define ODP_TIME_USEC_IN_NS 1000ULL
#define ODP_TIME_MSEC_IN_NS 1000000ULL
#define ODP_TIME_SEC_IN_NS  1000000000ULL
#define ODP_TIME_NULL ((odp_time_t){0})

odp_time_t odp_time_local(void);
odp_time_t odp_time_global(void);
uint64_t odp_time_local_ns(void);
uint64_t odp_time_global_ns(void);
odp_time_t odp_time_diff(odp_time_t t2, odp_time_t t1);
uint64_t odp_time_diff_ns(odp_time_t t2, odp_time_t t1);
odp_time_t odp_time_sum(odp_time_t t1, odp_time_t t2);
uint64_t odp_time_to_ns(odp_time_t time);
odp_time_t odp_time_local_from_ns(uint64_t ns);
int odp_time_cmp(odp_time_t t2, odp_time_t t1);
uint64_t odp_time_local_res(void);
void odp_time_wait_ns(uint64_t ns);

/* ------------------------------------------------------------ cpumask */
#define ODP_CPUMASK_SIZE 1024
#define ODP_CPUMASK_STR_SIZE ((ODP_CPUMASK_SIZE + 3) / 4 + 3)

typedef struct {
	uint64_t bits[ODP_CPUMASK_SIZE / 64];
} odp_cpumask_t;

void odp_cpumask_zero(odp_cpumask_t *mask);
void odp_cpumask_set(odp_cpumask_t *mask, int cpu);
void odp_cpumask_setall(odp_cpumask_t *mask);
void odp_cpumask_clr(odp_cpumask_t *mask, int cpu);
int odp_cpumask_isset(const odp_cpumask_t *mask, int cpu);
int odp_cpumask_count(const odp_cpumask_t *mask);
int odp_cpumask_first(const odp_cpumask_t *mask);
int odp_cpumask_last(const odp_cpumask_t *mask);
int odp_cpumask_next(const odp_cpumask_t *mask, int cpu);
void odp_cpumask_copy(odp_cpumask_t *dest, const odp_cpumask_t *src);
int32_t odp_cpumask_to_str(const odp_cpumask_t *mask, char *str, int32_t size);
void odp_cpumask_from_str(odp_cpumask_t *mask, const char *str);
int odp_cpumask_default_worker(odp_cpumask_t *mask, int num);
int odp_cpumask_default_control(odp_cpumask_t *mask, int num);
int odp_cpumask_all_available(odp_cpumask_t *mask);

/* ------------------------------------------------------------ init / threads */
typedef enum {
	ODP_THREAD_WORKER = 0,
	ODP_THREAD_CONTROL
} odp_thread_type_t;

typedef enum {
	ODP_MEM_MODEL_THREAD = 0,
	ODP_MEM_MODEL_PROCESS
} odp_mem_model_t;

typedef int (*odp_log_func_t)(int level, const char *fmt, ...);
typedef void (*odp_abort_func_t)(void);

typedef union odp_feature_t {
	struct {
		uint32_t cls      : 1;
		uint32_t compress : 1;
		uint32_t crypto   : 1;
		uint32_t dma      : 1;
		uint32_t ipsec    : 1;
		uint32_t ml       : 1;
		uint32_t schedule : 1;
		uint32_t stash    : 1;
		uint32_t time     : 1;
		uint32_t timer    : 1;
		uint32_t tm       : 1;
	} feat;
	uint32_t all_feat;
} odp_feature_t;

typedef struct odp_init_t {
	int num_worker;
	const odp_cpumask_t *worker_cpus;
	int num_control;
	const odp_cpumask_t *control_cpus;
	odp_log_func_t log_fn;
	odp_abort_func_t abort_fn;
	odp_mem_model_t mem_model;
	odp_feature_t not_used;
	uint64_t shm_max_memory;
	uint64_t shm_max_size;
} odp_init_t;

typedef struct odp_platform_init_t odp_platform_init_t;

void odp_init_param_init(odp_init_t *param);
int odp_init_global(odp_instance_t *instance, const odp_init_t *params,
		    const odp_platform_init_t *platform_params);
int odp_init_local(odp_instance_t instance, odp_thread_type_t thr_type);
int odp_term_local(void);
int odp_term_global(odp_instance_t instance);

int odp_thread_id(void);
int odp_thread_count(void);
int odp_thread_count_max(void);
odp_thread_type_t odp_thread_type(void);
int odp_cpu_id(void);
int odp_cpu_count(void);

void odp_sys_info_print(void);
uint64_t odp_sys_page_size(void);
int odp_sys_cache_line_size(void);
const char *odp_version_api_str(void);
const char *odp_version_impl_name(void);
const char *odp_version_impl_str(void);

/* ------------------------------------------------------------ shm */
#define ODP_SHM_SW_ONLY 0x0001
#define ODP_SHM_PROC    0x0002
#define ODP_SHM_EXPORT  0x0008
#define ODP_SHM_HP      0x0010
#define ODP_SHM_SINGLE_VA 0x0040

typedef struct odp_shm_info_t {
	const char *name;
	void *addr;
	uint64_t size;
	uint64_t page_size;
	uint32_t flags;
	uint32_t num_seg;
} odp_shm_info_t;

odp_shm_t odp_shm_reserve(const char *name, uint64_t size, uint64_t align, uint32_t flags);
int odp_shm_free(odp_shm_t shm);
odp_shm_t odp_shm_lookup(const char *name);
void *odp_shm_addr(odp_shm_t shm);
int odp_shm_info(odp_shm_t shm, odp_shm_info_t *info);
uint64_t odp_shm_to_u64(odp_shm_t shm);
void odp_shm_print_all(void);

/* ------------------------------------------------------------ events */
typedef enum odp_event_type_t {
	ODP_EVENT_BUFFER       = 1,
	ODP_EVENT_PACKET       = 2,
	ODP_EVENT_TIMEOUT      = 3,
	ODP_EVENT_IPSEC_STATUS = 5,
	ODP_EVENT_PACKET_VECTOR = 6,
	ODP_EVENT_PACKET_TX_COMPL = 7,
	ODP_EVENT_DMA_COMPL    = 8,
	ODP_EVENT_ML_COMPL     = 9,
	ODP_EVENT_VECTOR       = 10
} odp_event_type_t;

typedef enum odp_event_subtype_t {
	ODP_EVENT_NO_SUBTYPE = 0,
	ODP_EVENT_PACKET_BASIC,
	ODP_EVENT_PACKET_CRYPTO,
	ODP_EVENT_PACKET_IPSEC,
	ODP_EVENT_PACKET_COMP
} odp_event_subtype_t;

odp_event_type_t odp_event_type(odp_event_t event);
odp_event_subtype_t odp_event_subtype(odp_event_t event);
odp_event_type_t odp_event_types(odp_event_t event, odp_event_subtype_t *subtype);
void odp_event_free(odp_event_t event);
void odp_event_free_multi(const odp_event_t event[], int num);
odp_pool_t odp_event_pool(odp_event_t event);
int odp_event_is_valid(odp_event_t event);
uint64_t odp_event_to_u64(odp_event_t hdl);

/* event_vector.h */
odp_event_vector_t odp_event_vector_from_event(odp_event_t ev);
odp_event_t odp_event_vector_to_event(odp_event_vector_t evv);
odp_event_vector_t odp_event_vector_alloc(odp_pool_t pool);
void odp_event_vector_free(odp_event_vector_t evv);
uint32_t odp_event_vector_tbl(odp_event_vector_t evv, odp_event_t **event_tbl);
uint32_t odp_event_vector_size(odp_event_vector_t evv);
void odp_event_vector_size_set(odp_event_vector_t evv, uint32_t size);
odp_event_type_t odp_event_vector_type(odp_event_vector_t evv);
odp_pool_t odp_event_vector_pool(odp_event_vector_t evv);

/* packet.h: packet vectors (ODP_POOL_VECTOR pools, ODP_EVENT_PACKET_VECTOR
 * events); freeing a vector does not free its packets */
odp_packet_vector_t odp_packet_vector_from_event(odp_event_t ev);
odp_event_t odp_packet_vector_to_event(odp_packet_vector_t pktv);
odp_packet_vector_t odp_packet_vector_alloc(odp_pool_t pool);
void odp_packet_vector_free(odp_packet_vector_t pktv);
uint32_t odp_packet_vector_tbl(odp_packet_vector_t pktv, odp_packet_t **pkt_tbl);
uint32_t odp_packet_vector_size(odp_packet_vector_t pktv);
void odp_packet_vector_size_set(odp_packet_vector_t pktv, uint32_t size);
odp_pool_t odp_packet_vector_pool(odp_packet_vector_t pktv);
int odp_packet_vector_valid(odp_packet_vector_t pktv);

/* ------------------------------------------------------------ pools */
typedef enum odp_pool_type_t {
	ODP_POOL_BUFFER  = ODP_EVENT_BUFFER,
	ODP_POOL_PACKET  = ODP_EVENT_PACKET,
	ODP_POOL_TIMEOUT = ODP_EVENT_TIMEOUT,
	ODP_POOL_VECTOR  = ODP_EVENT_PACKET_VECTOR,
	ODP_POOL_DMA_COMPL,
	ODP_POOL_ML_COMPL,
	ODP_POOL_EVENT_VECTOR
} odp_pool_type_t;

typedef struct odp_pool_param_t {
	odp_pool_type_t type;
	struct {
		uint32_t num;
		uint32_t size;
		uint32_t align;
		uint32_t cache_size;
		uint32_t uarea_size;
	} buf;
	struct {
		uint32_t num;
		uint32_t max_num;
		uint32_t len;
		uint32_t max_len;
		uint32_t seg_len;
		uint32_t align;
		uint32_t uarea_size;
		uint32_t headroom;
		uint32_t num_subparam;
		uint32_t sub[7];
		uint32_t cache_size;
	} pkt;
	struct {
		uint32_t num;
		uint32_t uarea_size;
		uint32_t cache_size;
	} tmo;
	struct {
		uint32_t num;
		uint32_t max_size;
		uint32_t uarea_size;
		uint32_t cache_size;
	} vector;
	struct {
		uint32_t num;
		uint32_t max_size;
		uint32_t uarea_size;
		uint32_t cache_size;
	} event_vector;
	void *uarea_init_arg;
	void (*uarea_init)(void *uarea, uint32_t size, void *args, uint32_t index);
} odp_pool_param_t;

typedef struct odp_pool_info_t {
	odp_pool_type_t type;
	const char *name;
	odp_pool_param_t params;
	uint64_t min_data_addr;
	uint64_t max_data_addr;
} odp_pool_info_t;

typedef struct odp_pool_capability_t {
	uint32_t max_pools;
	struct {
		uint32_t max_pools;
		uint32_t max_len;
		uint32_t max_num;
		uint32_t max_headroom;
		uint32_t min_headroom;
		uint32_t max_segs_per_pkt;
		uint32_t min_seg_len;
		uint32_t max_seg_len;
		uint32_t max_uarea_size;
	} pkt;
	struct {
		uint32_t max_pools;
		uint32_t max_num;
		uint32_t max_size;
	} event_vector;
} odp_pool_capability_t;

void odp_pool_param_init(odp_pool_param_t *param);
int odp_pool_capability(odp_pool_capability_t *capa);
odp_pool_t odp_pool_create(const char *name, const odp_pool_param_t *param);
int odp_pool_destroy(odp_pool_t pool);
odp_pool_t odp_pool_lookup(const char *name);
int odp_pool_info(odp_pool_t pool, odp_pool_info_t *info);
void odp_pool_print(odp_pool_t pool);
void odp_pool_print_all(void);
uint64_t odp_pool_to_u64(odp_pool_t hdl);
int odp_pool_index(odp_pool_t pool);
unsigned int odp_pool_max_index(void);

/* ------------------------------------------------------------ packets */
typedef enum odp_proto_layer_t {
	ODP_PROTO_LAYER_NONE = 0,
	ODP_PROTO_LAYER_L2,
	ODP_PROTO_LAYER_L3,
	ODP_PROTO_LAYER_L4,
	ODP_PROTO_LAYER_ALL
} odp_proto_layer_t;

odp_packet_t odp_packet_alloc(odp_pool_t pool, uint32_t len);
int odp_packet_alloc_multi(odp_pool_t pool, uint32_t len, odp_packet_t pkt[], int num);
void odp_packet_free(odp_packet_t pkt);
void odp_packet_free_multi(const odp_packet_t pkt[], int num);
odp_packet_t odp_packet_from_event(odp_event_t ev);
void odp_packet_from_event_multi(odp_packet_t pkt[], const odp_event_t ev[], int num);
odp_event_t odp_packet_to_event(odp_packet_t pkt);
void odp_packet_to_event_multi(const odp_packet_t pkt[], odp_event_t ev[], int num);
uint32_t odp_packet_len(odp_packet_t pkt);
uint32_t odp_packet_seg_len(odp_packet_t pkt);
uint32_t odp_packet_buf_len(odp_packet_t pkt);
uint32_t odp_packet_headroom(odp_packet_t pkt);
uint32_t odp_packet_tailroom(odp_packet_t pkt);
void *odp_packet_data(odp_packet_t pkt);
void *odp_packet_head(odp_packet_t pkt);
void *odp_packet_tail(odp_packet_t pkt);
void *odp_packet_offset(odp_packet_t pkt, uint32_t offset, uint32_t *len, void *seg);
void *odp_packet_push_head(odp_packet_t pkt, uint32_t len);
void *odp_packet_pull_head(odp_packet_t pkt, uint32_t len);
void *odp_packet_push_tail(odp_packet_t pkt, uint32_t len);
void *odp_packet_pull_tail(odp_packet_t pkt, uint32_t len);
odp_pool_t odp_packet_pool(odp_packet_t pkt);
odp_pktio_t odp_packet_input(odp_packet_t pkt);
int odp_packet_input_index(odp_packet_t pkt);
int odp_packet_copy_to_mem(odp_packet_t pkt, uint32_t offset, uint32_t len, void *dst);
int odp_packet_copy_from_mem(odp_packet_t pkt, uint32_t offset, uint32_t len, const void *src);
odp_packet_t odp_packet_copy(odp_packet_t pkt, odp_pool_t pool);
int odp_packet_is_valid(odp_packet_t pkt);
void odp_packet_print(odp_packet_t pkt);
void odp_packet_print_data(odp_packet_t pkt, uint32_t offset, uint32_t len);
uint64_t odp_packet_to_u64(odp_packet_t hdl);
void *odp_packet_user_ptr(odp_packet_t pkt);
void odp_packet_user_ptr_set(odp_packet_t pkt, const void *user_ptr);
int odp_packet_num_segs(odp_packet_t pkt);
int odp_packet_is_segmented(odp_packet_t pkt);

/* layer offsets / pointers (packet.h) */
void *odp_packet_l2_ptr(odp_packet_t pkt, uint32_t *len);
uint32_t odp_packet_l2_offset(odp_packet_t pkt);
int odp_packet_l2_offset_set(odp_packet_t pkt, uint32_t offset);
void *odp_packet_l3_ptr(odp_packet_t pkt, uint32_t *len);
uint32_t odp_packet_l3_offset(odp_packet_t pkt);
int odp_packet_l3_offset_set(odp_packet_t pkt, uint32_t offset);
void *odp_packet_l4_ptr(odp_packet_t pkt, uint32_t *len);
uint32_t odp_packet_l4_offset(odp_packet_t pkt);
int odp_packet_l4_offset_set(odp_packet_t pkt, uint32_t offset);

/* classifier metadata (packet.h: odp_packet_cls_mark) */
uint64_t odp_packet_cls_mark(odp_packet_t pkt);

/* packet_flags.h */
int odp_packet_has_error(odp_packet_t pkt);
int odp_packet_has_l2_error(odp_packet_t pkt);
int odp_packet_has_l3_error(odp_packet_t pkt);
int odp_packet_has_l4_error(odp_packet_t pkt);

/* Checksum check status (include/odp/api/spec/packet_types.h, values from
 * the receive parse with pktin checksum options, packet_inlines.h:389-420) */
typedef enum {
	ODP_PACKET_CHKSUM_UNKNOWN = 0,
	ODP_PACKET_CHKSUM_BAD,
	ODP_PACKET_CHKSUM_OK
} odp_packet_chksum_status_t;

odp_packet_chksum_status_t odp_packet_l3_chksum_status(odp_packet_t pkt);
odp_packet_chksum_status_t odp_packet_l4_chksum_status(odp_packet_t pkt);
int odp_packet_has_l2(odp_packet_t pkt);
int odp_packet_has_l3(odp_packet_t pkt);
int odp_packet_has_l4(odp_packet_t pkt);
int odp_packet_has_eth(odp_packet_t pkt);
int odp_packet_has_eth_bcast(odp_packet_t pkt);
int odp_packet_has_eth_mcast(odp_packet_t pkt);
int odp_packet_has_jumbo(odp_packet_t pkt);
int odp_packet_has_vlan(odp_packet_t pkt);
int odp_packet_has_vlan_qinq(odp_packet_t pkt);
int odp_packet_has_arp(odp_packet_t pkt);
int odp_packet_has_ipv4(odp_packet_t pkt);
int odp_packet_has_ipv6(odp_packet_t pkt);
int odp_packet_has_ip_bcast(odp_packet_t pkt);
int odp_packet_has_ip_mcast(odp_packet_t pkt);
int odp_packet_has_ipfrag(odp_packet_t pkt);
int odp_packet_has_ipopt(odp_packet_t pkt);
int odp_packet_has_ipsec(odp_packet_t pkt);
int odp_packet_has_udp(odp_packet_t pkt);
int odp_packet_has_tcp(odp_packet_t pkt);
int odp_packet_has_sctp(odp_packet_t pkt);
int odp_packet_has_icmp(odp_packet_t pkt);
int odp_packet_has_flow_hash(odp_packet_t pkt);
int odp_packet_has_ts(odp_packet_t pkt);

/* ------------------------------------------------------------ queues */
typedef enum odp_queue_type_t {
	ODP_QUEUE_TYPE_PLAIN = 0,
	ODP_QUEUE_TYPE_SCHED,
	ODP_QUEUE_TYPE_AGGR     /* event aggregator of a queue (odp_queue_aggr) */
} odp_queue_type_t;

typedef enum odp_queue_op_mode_t {
	ODP_QUEUE_OP_MT = 0,
	ODP_QUEUE_OP_MT_UNSAFE,
	ODP_QUEUE_OP_DISABLED
} odp_queue_op_mode_t;

typedef enum odp_nonblocking_t {
	ODP_BLOCKING = 0,
	ODP_NONBLOCKING_LF,
	ODP_NONBLOCKING_WF
} odp_nonblocking_t;

typedef enum odp_queue_order_t {
	ODP_QUEUE_ORDER_KEEP = 0,
	ODP_QUEUE_ORDER_IGNORE
} odp_queue_order_t;

typedef int odp_schedule_prio_t;
typedef int odp_schedule_sync_t;
typedef int odp_schedule_group_t;

#define ODP_SCHED_WAIT     UINT64_MAX
#define ODP_SCHED_NO_WAIT  0
#define ODP_SCHED_SYNC_PARALLEL 0
#define ODP_SCHED_SYNC_ATOMIC   1
#define ODP_SCHED_SYNC_ORDERED  2
#define ODP_SCHED_GROUP_INVALID ((odp_schedule_group_t)-1)
#define ODP_SCHED_GROUP_ALL     0
#define ODP_SCHED_GROUP_WORKER  1
#define ODP_SCHED_GROUP_CONTROL 2
#define ODP_SCHED_GROUP_NAME_LEN 32
#define ODP_SCHED_MAX_PRIOS 8

typedef struct odp_schedule_param_t {
	odp_schedule_prio_t prio;
	odp_schedule_sync_t sync;
	odp_schedule_group_t group;
	uint32_t lock_count;
} odp_schedule_param_t;

typedef struct odp_event_aggr_config_t {
	odp_pool_t pool;
	uint64_t max_tmo_ns;
	uint32_t max_size;
	odp_event_type_t event_type;
} odp_event_aggr_config_t;

typedef struct odp_queue_param_t {
	odp_queue_type_t type;
	odp_queue_op_mode_t enq_mode;
	odp_queue_op_mode_t deq_mode;
	odp_schedule_param_t sched;
	odp_queue_order_t order;
	odp_nonblocking_t nonblocking;
	void *context;
	uint32_t context_len;
	uint32_t size;
	uint32_t num_aggr;
	const odp_event_aggr_config_t *aggr;
} odp_queue_param_t;

typedef struct odp_queue_info_t {
	const char *name;
	odp_queue_type_t type;
	odp_queue_param_t param;
	odp_event_aggr_config_t aggr_config;
} odp_queue_info_t;

typedef struct odp_queue_capability_t {
	uint32_t max_queues;
	struct {
		uint32_t max_num;
		uint32_t max_size;
	} plain;
} odp_queue_capability_t;

typedef struct odp_aggr_enq_profile_t {
	enum {
		ODP_AEP_TYPE_NONE,
		ODP_AEP_TYPE_IPV4_FRAG,
		ODP_AEP_TYPE_IPV6_FRAG,
		ODP_AEP_TYPE_CUSTOM,
	} type;
	uintptr_t param;
} odp_aggr_enq_profile_t;

void odp_queue_param_init(odp_queue_param_t *param);
int odp_queue_capability(odp_queue_capability_t *capa);
odp_queue_t odp_queue_create(const char *name, const odp_queue_param_t *param);
int odp_queue_destroy(odp_queue_t queue);
odp_queue_t odp_queue_lookup(const char *name);
odp_queue_t odp_queue_aggr(odp_queue_t queue, uint32_t aggr_index);
int odp_queue_enq(odp_queue_t queue, odp_event_t ev);
int odp_queue_enq_multi(odp_queue_t queue, const odp_event_t events[], int num);
odp_event_t odp_queue_deq(odp_queue_t queue);
int odp_queue_deq_multi(odp_queue_t queue, odp_event_t events[], int num);
odp_queue_type_t odp_queue_type(odp_queue_t queue);
odp_schedule_sync_t odp_queue_sched_type(odp_queue_t queue);
odp_schedule_prio_t odp_queue_sched_prio(odp_queue_t queue);
int odp_queue_context_set(odp_queue_t queue, void *context, uint32_t len);
void *odp_queue_context(odp_queue_t queue);
int odp_queue_info(odp_queue_t queue, odp_queue_info_t *info);
void odp_queue_print(odp_queue_t queue);
void odp_queue_print_all(void);
uint64_t odp_queue_to_u64(odp_queue_t hdl);

/* ------------------------------------------------------------ scheduler */
typedef struct odp_schedule_config_t {
	uint32_t num_queues;
	uint32_t queue_size;
	uint32_t max_flow_id;
	struct {
		odp_bool_t all;
		odp_bool_t control;
		odp_bool_t worker;
	} sched_group;
} odp_schedule_config_t;

void odp_schedule_config_init(odp_schedule_config_t *config);
int odp_schedule_config(const odp_schedule_config_t *config);
uint64_t odp_schedule_wait_time(uint64_t ns);
odp_event_t odp_schedule(odp_queue_t *from, uint64_t wait);
int odp_schedule_multi(odp_queue_t *from, uint64_t wait, odp_event_t events[], int num);
int odp_schedule_multi_wait(odp_queue_t *from, odp_event_t events[], int num);
int odp_schedule_multi_no_wait(odp_queue_t *from, odp_event_t events[], int num);
void odp_schedule_pause(void);
void odp_schedule_resume(void);
void odp_schedule_release_atomic(void);
void odp_schedule_release_ordered(void);
int odp_schedule_min_prio(void);
int odp_schedule_max_prio(void);
int odp_schedule_default_prio(void);
int odp_schedule_num_prio(void);

/* ------------------------------------------------------------ packet I/O */
typedef struct { _odp_pktin_hdl_t q; int index; odp_pktio_t pktio; } odp_pktin_queue_t;
typedef struct { void *q; int index; odp_pktio_t pktio; } odp_pktout_queue_t;

typedef enum odp_pktin_mode_t {
	ODP_PKTIN_MODE_DIRECT = 0,
	ODP_PKTIN_MODE_SCHED,
	ODP_PKTIN_MODE_QUEUE,
	ODP_PKTIN_MODE_DISABLED
} odp_pktin_mode_t;

typedef enum odp_pktout_mode_t {
	ODP_PKTOUT_MODE_DIRECT = 0,
	ODP_PKTOUT_MODE_QUEUE,
	ODP_PKTOUT_MODE_TM,
	ODP_PKTOUT_MODE_DISABLED
} odp_pktout_mode_t;

typedef enum odp_pktio_op_mode_t {
	ODP_PKTIO_OP_MT = 0,
	ODP_PKTIO_OP_MT_UNSAFE
} odp_pktio_op_mode_t;

/* packet_io_types.h:124-146 */
typedef union odp_pktin_hash_proto_t {
	struct {
		uint32_t ipv4_udp : 1;
		uint32_t ipv4_tcp : 1;
		uint32_t ipv4     : 1;
		uint32_t ipv6_udp : 1;
		uint32_t ipv6_tcp : 1;
		uint32_t ipv6     : 1;
	} proto;
	uint32_t all_bits;
} odp_pktin_hash_proto_t;

typedef struct odp_pktin_vector_config_t {
	odp_bool_t enable;
	odp_pool_t pool;
	uint64_t max_tmo_ns;
	uint32_t max_size;
} odp_pktin_vector_config_t;

typedef struct odp_pktin_queue_param_ovr_t {
	odp_schedule_group_t group;
} odp_pktin_queue_param_ovr_t;

typedef struct odp_pktin_queue_param_t {
	odp_pktio_op_mode_t op_mode;
	odp_bool_t classifier_enable;
	odp_bool_t hash_enable;
	odp_pktin_hash_proto_t hash_proto;
	uint32_t num_queues;
	uint32_t queue_size[ODP_PKTIN_MAX_QUEUES];
	odp_queue_param_t queue_param;
	odp_pktin_queue_param_ovr_t *queue_param_ovr;
	odp_pktin_vector_config_t vector;
} odp_pktin_queue_param_t;

typedef struct odp_pktout_queue_param_t {
	odp_pktio_op_mode_t op_mode;
	uint32_t num_queues;
	uint32_t queue_size[ODP_PKTOUT_MAX_QUEUES];
} odp_pktout_queue_param_t;

typedef struct odp_pktio_param_t {
	odp_pktin_mode_t in_mode;
	odp_pktout_mode_t out_mode;
} odp_pktio_param_t;

typedef union odp_pktin_config_opt_t {
	struct {
		uint64_t ts_all        : 1;
		uint64_t ts_ptp        : 1;
		uint64_t ipv4_chksum   : 1;
		uint64_t udp_chksum    : 1;
		uint64_t tcp_chksum    : 1;
		uint64_t sctp_chksum   : 1;
		uint64_t drop_ipv4_err : 1;
		uint64_t drop_ipv6_err : 1;
		uint64_t drop_udp_err  : 1;
		uint64_t drop_tcp_err  : 1;
		uint64_t drop_sctp_err : 1;
	} bit;
	uint64_t all_bits;
} odp_pktin_config_opt_t;

typedef union odp_pktout_config_opt_t {
	struct {
		uint64_t ts_ena          : 1;
		uint64_t ipv4_chksum_ena : 1;
		uint64_t udp_chksum_ena  : 1;
		uint64_t tcp_chksum_ena  : 1;
		uint64_t sctp_chksum_ena : 1;
		uint64_t ipv4_chksum     : 1;
		uint64_t udp_chksum      : 1;
		uint64_t tcp_chksum      : 1;
		uint64_t sctp_chksum     : 1;
		uint64_t no_packet_refs  : 1;
		uint64_t aging_ena       : 1;
		uint64_t proto_stats_ena : 1;
	} bit;
	uint64_t all_bits;
} odp_pktout_config_opt_t;

typedef struct odp_pktio_parser_config_t {
	odp_proto_layer_t layer;
} odp_pktio_parser_config_t;

typedef enum odp_pktio_link_pause_t {
	ODP_PKTIO_LINK_PAUSE_UNKNOWN = -1,
	ODP_PKTIO_LINK_PAUSE_OFF = 0,
	ODP_PKTIO_LINK_PAUSE_ON = 1,
	ODP_PKTIO_LINK_PFC_ON = 2
} odp_pktio_link_pause_t;

typedef struct odp_reass_config_t {
	odp_bool_t en_ipv4;
	odp_bool_t en_ipv6;
	uint32_t max_wait_time;
	uint8_t max_num_frags;
} odp_reass_config_t;

typedef struct odp_pktio_config_t {
	odp_pktin_config_opt_t pktin;
	odp_pktout_config_opt_t pktout;
	odp_pktio_parser_config_t parser;
	odp_bool_t enable_loop;
	odp_bool_t inbound_ipsec;
	odp_bool_t outbound_ipsec;
	odp_bool_t enable_lso;
	odp_reass_config_t reassembly;
	struct {
		odp_pktio_link_pause_t pause_rx;
		odp_pktio_link_pause_t pause_tx;
	} flow_control;
	struct {
		uint32_t mode_event : 1;
		uint32_t mode_poll : 1;
		uint32_t max_compl_id;
	} tx_compl;
} odp_pktio_config_t;

typedef union odp_pktio_set_op_t {
	struct {
		uint32_t promisc_mode : 1;
		uint32_t mac_addr : 1;
		uint32_t skip_offset : 1;
		uint32_t maxlen : 1;
	} op;
	uint32_t all_bits;
} odp_pktio_set_op_t;

typedef struct odp_pktio_capability_t {
	uint32_t max_input_queues;
	uint32_t min_input_queue_size;
	uint32_t max_input_queue_size;
	uint32_t max_output_queues;
	uint32_t min_output_queue_size;
	uint32_t max_output_queue_size;
	odp_pktio_config_t config;
	odp_pktio_set_op_t set_op;
	struct {
		odp_bool_t equal;
		uint32_t min_input;
		uint32_t max_input;
		uint32_t min_output;
		uint32_t max_output;
	} maxlen;
	odp_support_t loop_supported;
	odp_bool_t vector_supported;
} odp_pktio_capability_t;

typedef struct odp_pktio_stats_t {
	uint64_t in_octets;
	uint64_t in_packets;
	uint64_t in_ucast_pkts;
	uint64_t in_mcast_pkts;
	uint64_t in_bcast_pkts;
	uint64_t in_discards;
	uint64_t in_errors;
	uint64_t out_octets;
	uint64_t out_packets;
	uint64_t out_ucast_pkts;
	uint64_t out_mcast_pkts;
	uint64_t out_bcast_pkts;
	uint64_t out_discards;
	uint64_t out_errors;
} odp_pktio_stats_t;

typedef struct odp_pktio_info_t {
	const char *name;
	const char *drv_name;
	odp_pool_t pool;
	odp_pktio_param_t param;
} odp_pktio_info_t;

#define ODP_PKTIN_NO_WAIT 0
#define ODP_PKTIN_WAIT    UINT64_MAX

void odp_pktio_param_init(odp_pktio_param_t *param);
void odp_pktin_queue_param_init(odp_pktin_queue_param_t *param);
void odp_pktout_queue_param_init(odp_pktout_queue_param_t *param);
void odp_pktio_config_init(odp_pktio_config_t *config);
odp_pktio_t odp_pktio_open(const char *name, odp_pool_t pool, const odp_pktio_param_t *param);
int odp_pktio_capability(odp_pktio_t pktio, odp_pktio_capability_t *capa);
int odp_pktio_config(odp_pktio_t pktio, const odp_pktio_config_t *config);
int odp_pktin_queue_config(odp_pktio_t pktio, const odp_pktin_queue_param_t *param);
int odp_pktout_queue_config(odp_pktio_t pktio, const odp_pktout_queue_param_t *param);
int odp_pktin_queue(odp_pktio_t pktio, odp_pktin_queue_t queues[], int num);
int odp_pktin_event_queue(odp_pktio_t pktio, odp_queue_t queues[], int num);
int odp_pktout_queue(odp_pktio_t pktio, odp_pktout_queue_t queues[], int num);
int odp_pktio_start(odp_pktio_t pktio);
int odp_pktio_stop(odp_pktio_t pktio);
int odp_pktio_close(odp_pktio_t pktio);
odp_pktio_t odp_pktio_lookup(const char *name);
int odp_pktin_recv(odp_pktin_queue_t queue, odp_packet_t packets[], int num);
int odp_pktin_recv_tmo(odp_pktin_queue_t queue, odp_packet_t packets[], int num, uint64_t wait);
uint64_t odp_pktin_wait_time(uint64_t nsec);
int odp_pktout_send(odp_pktout_queue_t queue, const odp_packet_t packets[], int num);
int odp_pktio_promisc_mode(odp_pktio_t pktio);
int odp_pktio_promisc_mode_set(odp_pktio_t pktio, odp_bool_t enable);
int odp_pktio_mac_addr(odp_pktio_t pktio, void *mac_addr, int size);
uint32_t odp_pktio_mtu(odp_pktio_t pktio);
int odp_pktio_stats(odp_pktio_t pktio, odp_pktio_stats_t *stats);
int odp_pktio_stats_reset(odp_pktio_t pktio);
int odp_pktio_info(odp_pktio_t pktio, odp_pktio_info_t *info);
int odp_pktio_index(odp_pktio_t pktio);
void odp_pktio_print(odp_pktio_t pktio);
uint64_t odp_pktio_to_u64(odp_pktio_t pktio);

/* ------------------------------------------------------------ build extensions */
/* 1 when a pktio has no more input and no receive burst in flight (pcap past
 * EOF, loop queue empty), 0 otherwise, -1 on a bad handle. */
int odp_amd_pktio_rx_idle(odp_pktio_t pktio);

#ifdef __cplusplus
}
#endif

#endif /* ODP_AMD_RT_H_ */
