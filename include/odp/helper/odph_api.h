/*
 * odph_api.h -- the ODP helper subset (libodph.so) the classifier example
 * uses: command-line helper options, thread create/join over pthreads,
 * address parsers, protocol header structs and the log macros.
 *
 * Follows helper/include/odp/helper/{threads.h, eth.h, ip.h, string.h,
 * debug.h, macros.h} of the reference: same names, field paths and return
 * conventions (0 / -1; odph_ipv4_addr_parse returns a host-order address,
 * helper/ip.c:10-28).
 */
#ifndef ODPH_AMD_API_H_
#define ODPH_AMD_API_H_

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>

#include "../../odp_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------ macros */
#define ODPH_MIN(a, b) __extension__ ({ __typeof__(a) _a = (a); __typeof__(b) _b = (b); _a < _b ? _a : _b; })
#define ODPH_MAX(a, b) __extension__ ({ __typeof__(a) _a = (a); __typeof__(b) _b = (b); _a > _b ? _a : _b; })
#define ODPH_ARRAY_SIZE(x) (sizeof(x) / sizeof((x)[0]))

/* debug.h: the helper logs to stderr with the call site, ODPH_ABORT aborts */
#define ODPH_ERR(fmt, ...) \
	fprintf(stderr, "%s:%d:%s(): " fmt, __FILE__, __LINE__, __func__, ##__VA_ARGS__)
#define ODPH_DBG(fmt, ...) do { } while (0)
#define ODPH_ABORT(fmt, ...) \
	do { ODPH_ERR(fmt, ##__VA_ARGS__); abort(); } while (0)
#define ODPH_ASSERT(cond) do { if (!(cond)) ODPH_ABORT("%s\n", #cond); } while (0)

/* string.h */
static inline char *odph_strcpy(char *dst, const char *src, size_t sz)
{
	if (!sz)
		return dst;
	size_t n = strnlen(src, sz - 1);

	memcpy(dst, src, n);
	dst[n] = 0;
	return dst;
}

/* ------------------------------------------------------------ protocols */
#define ODPH_ETHADDR_LEN     6
#define ODPH_ETHHDR_LEN      14
#define ODPH_VLANHDR_LEN     4
#define ODPH_ETH_LEN_MIN     60
#define ODPH_ETH_LEN_MAX     1514
#define ODPH_ETHTYPE_IPV4    0x0800
#define ODPH_ETHTYPE_ARP     0x0806
#define ODPH_ETHTYPE_VLAN    0x8100
#define ODPH_ETHTYPE_VLAN_OUTER 0x88A8
#define ODPH_ETHTYPE_IPV6    0x86dd
#define ODPH_IPV4            4
#define ODPH_IPV4HDR_LEN     20
#define ODPH_IPV6HDR_LEN     40
#define ODPH_IPPROTO_ICMPV4  0x01
#define ODPH_IPPROTO_TCP     0x06
#define ODPH_IPPROTO_UDP     0x11
#define ODPH_IPPROTO_SCTP    0x84
#define ODPH_UDPHDR_LEN      8
#define ODPH_TCPHDR_LEN      20

typedef struct __attribute__((packed)) {
	uint8_t addr[ODPH_ETHADDR_LEN];
} odph_ethaddr_t;

typedef struct __attribute__((packed)) {
	odph_ethaddr_t dst;
	odph_ethaddr_t src;
	odp_u16be_t type;
} odph_ethhdr_t;

typedef struct __attribute__((packed)) {
	odp_u16be_t tci;
	odp_u16be_t type;
} odph_vlanhdr_t;

typedef struct __attribute__((packed)) {
	uint8_t ver_ihl;
	uint8_t tos;
	odp_u16be_t tot_len;
	odp_u16be_t id;
	odp_u16be_t frag_offset;
	uint8_t ttl;
	uint8_t proto;
	odp_u16sum_t chksum;
	odp_u32be_t src_addr;
	odp_u32be_t dst_addr;
} odph_ipv4hdr_t;

typedef struct __attribute__((packed)) {
	odp_u32be_t ver_tc_flow;
	odp_u16be_t payload_len;
	uint8_t next_hdr;
	uint8_t hop_limit;
	uint8_t src_addr[16];
	uint8_t dst_addr[16];
} odph_ipv6hdr_t;

typedef struct __attribute__((packed)) {
	odp_u16be_t src_port;
	odp_u16be_t dst_port;
	odp_u16be_t length;
	odp_u16be_t chksum;
} odph_udphdr_t;

typedef struct __attribute__((packed)) {
	odp_u16be_t src_port;
	odp_u16be_t dst_port;
	odp_u32be_t seq_no;
	odp_u32be_t ack_no;
	uint16_t hl_flags;
	odp_u16be_t window;
	odp_u16be_t cksm;
	odp_u16be_t urgptr;
} odph_tcphdr_t;

/* "a.b.c.d" -> host-order u32; 0 / -1 (helper/ip.c) */
int odph_ipv4_addr_parse(uint32_t *ip_addr, const char *str);
/* "xx:xx:xx:xx:xx:xx" -> mac; 0 / -1 (helper/eth.c) */
int odph_eth_addr_parse(odph_ethaddr_t *mac, const char *str);

/* ------------------------------------------------------------ threads */
typedef struct {
	int (*start)(void *arg);
	void *arg;
	odp_thread_type_t thr_type;
	uint64_t stack_size;
} odph_thread_param_t;

typedef struct {
	uint32_t status;
	odp_atomic_u32_t *init_status;
	odp_mem_model_t mem_model;
	odp_instance_t instance;
	odph_thread_param_t thr_params;
} odph_thread_start_args_t;

typedef struct {
	odph_thread_start_args_t start_args;
	int cpu;
	uint8_t last;
	union {
		struct {
			pthread_t thread_id;
			pthread_attr_t attr;
		} thread;
		struct {
			pid_t pid;
			int status;
		} proc;
	};
} odph_thread_t;

typedef struct {
	odp_mem_model_t mem_model;
} odph_helper_options_t;

typedef struct {
	odp_instance_t instance;
	const odp_cpumask_t *cpumask;
	int thread_model;
	int sync;
	uint64_t sync_timeout;
	int share_param;
} odph_thread_common_param_t;

typedef struct {
	odp_bool_t is_sig;
	int ret;
} odph_thread_join_result_t;

void odph_thread_param_init(odph_thread_param_t *param);
void odph_thread_common_param_init(odph_thread_common_param_t *param);
int odph_thread_create(odph_thread_t thread[], const odph_thread_common_param_t *param,
		       const odph_thread_param_t thr_param[], int num);
int odph_thread_join(odph_thread_t thread[], int num);
int odph_thread_join_result(odph_thread_t thread[], odph_thread_join_result_t res[], int num);
int odph_odpthread_setaffinity(const int cpu);
int odph_odpthread_getaffinity(void);
int odph_parse_options(int argc, char *argv[]);
int odph_options(odph_helper_options_t *options);

#ifdef __cplusplus
}
#endif

#endif /* ODPH_AMD_API_H_ */
