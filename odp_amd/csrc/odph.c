/*
 * odph.c -- the ODP helper subset (libodph.so): helper options, threads over
 * pthreads, IPv4 / MAC address parsers.
 *
 * Behaviour follows helper/threads.c (odph_thread_create runs the start
 * function in a new pthread after odp_init_local() of the given thread type,
 * pinned to the next CPU of the mask; odph_thread_join returns the number of
 * threads joined), helper/ip.c:10-28 (odph_ipv4_addr_parse: dotted quad ->
 * host-order u32, each part 0-255) and helper/eth.c (six ':'-separated hex
 * bytes).  Process mode (--odph_proc) is not supported by this build: the
 * option parses, and thread creation fails loudly if it is selected.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "odp/helper/odph_api.h"

static odph_helper_options_t helper_opts = { .mem_model = ODP_MEM_MODEL_THREAD };

/* Consumes the helper's own --odph_* options and returns the new argc
 * (helper/threads.c odph_parse_options). */
int odph_parse_options(int argc, char *argv[])
{
	int i, j = 1;

	for (i = 1; i < argc; i++) {
		if (strcmp(argv[i], "--odph_proc") == 0) {
			helper_opts.mem_model = ODP_MEM_MODEL_PROCESS;
			continue;
		}
		if (strcmp(argv[i], "--odph_thread") == 0) {
			helper_opts.mem_model = ODP_MEM_MODEL_THREAD;
			continue;
		}
		argv[j++] = argv[i];
	}
	if (j < argc)
		argv[j] = NULL;
	return j;
}

int odph_options(odph_helper_options_t *options)
{
	if (!options)
		return -1;
	*options = helper_opts;
	return 0;
}

void odph_thread_param_init(odph_thread_param_t *p)
{
	memset(p, 0, sizeof(*p));
}

void odph_thread_common_param_init(odph_thread_common_param_t *p)
{
	memset(p, 0, sizeof(*p));
	p->sync_timeout = ODP_TIME_SEC_IN_NS;
}

static void *thread_run(void *arg)
{
	odph_thread_t *t = arg;
	odph_thread_start_args_t *a = &t->start_args;

	if (t->cpu >= 0)
		(void)odph_odpthread_setaffinity(t->cpu);
	if (odp_init_local(a->instance, a->thr_params.thr_type)) {
		ODPH_ERR("Local init failed\n");
		return (void *)(intptr_t)-1;
	}
	int ret = a->thr_params.start(a->thr_params.arg);

	if (odp_term_local() < 0)
		ODPH_ERR("Local term failed\n");
	return (void *)(intptr_t)ret;
}

int odph_thread_create(odph_thread_t thread[], const odph_thread_common_param_t *param,
		       const odph_thread_param_t thr_param[], int num)
{
	int cpu, i;

	if (!param || !thr_param || num <= 0)
		return -1;
	if (helper_opts.mem_model == ODP_MEM_MODEL_PROCESS || param->thread_model == 1) {
		ODPH_ERR("process mode threads are not supported by this build\n");
		return -1;
	}
	cpu = param->cpumask ? odp_cpumask_first(param->cpumask) : -1;
	for (i = 0; i < num; i++) {
		odph_thread_t *t = &thread[i];
		const odph_thread_param_t *tp = param->share_param ? &thr_param[0] : &thr_param[i];

		memset(t, 0, sizeof(*t));
		t->cpu = cpu;
		t->start_args.mem_model = ODP_MEM_MODEL_THREAD;
		t->start_args.instance = param->instance;
		t->start_args.thr_params = *tp;
		pthread_attr_init(&t->thread.attr);
		if (tp->stack_size)
			pthread_attr_setstacksize(&t->thread.attr, (size_t)tp->stack_size);
		if (pthread_create(&t->thread.thread_id, &t->thread.attr, thread_run, t)) {
			ODPH_ERR("Failed to start thread on CPU %d\n", cpu);
			pthread_attr_destroy(&t->thread.attr);
			break;
		}
		t->start_args.status = 1;
		if (param->cpumask) {
			cpu = odp_cpumask_next(param->cpumask, cpu);
			if (cpu < 0)
				cpu = odp_cpumask_first(param->cpumask);
		}
	}
	if (i > 0)
		thread[i - 1].last = 1;
	return i;
}

int odph_thread_join_result(odph_thread_t thread[], odph_thread_join_result_t res[], int num)
{
	int i;

	for (i = 0; i < num; i++) {
		void *rv = NULL;

		if (!thread[i].start_args.status)
			break;
		if (pthread_join(thread[i].thread.thread_id, &rv)) {
			ODPH_ERR("Failed to join thread %d\n", i);
			break;
		}
		pthread_attr_destroy(&thread[i].thread.attr);
		thread[i].start_args.status = 0;
		if (res) {
			res[i].is_sig = 0;
			res[i].ret = (int)(intptr_t)rv;
		}
	}
	return i;
}

int odph_thread_join(odph_thread_t thread[], int num)
{
	return odph_thread_join_result(thread, NULL, num);
}

int odph_odpthread_setaffinity(const int cpu)
{
	cpu_set_t s;

	CPU_ZERO(&s);
	CPU_SET(cpu, &s);
	return pthread_setaffinity_np(pthread_self(), sizeof(s), &s) ? -1 : 0;
}

int odph_odpthread_getaffinity(void)
{
	cpu_set_t s;

	if (pthread_getaffinity_np(pthread_self(), sizeof(s), &s))
		return -1;
	for (int c = 0; c < CPU_SETSIZE; c++)
		if (CPU_ISSET(c, &s))
			return c;
	return -1;
}

/* helper/ip.c:10-28 */
int odph_ipv4_addr_parse(uint32_t *ip_addr, const char *str)
{
	unsigned int b[4] = { 0, 0, 0, 0 };

	if (!ip_addr || !str)
		return -1;
	/* trailing characters are ignored, as in the reference's sscanf */
	if (sscanf(str, "%u.%u.%u.%u", &b[0], &b[1], &b[2], &b[3]) != 4)
		return -1;
	for (int i = 0; i < 4; i++)
		if (b[i] > 255)
			return -1;
	*ip_addr = b[0] << 24 | b[1] << 16 | b[2] << 8 | b[3];
	return 0;
}

/* helper/eth.c: "xx:xx:xx:xx:xx:xx" */
int odph_eth_addr_parse(odph_ethaddr_t *mac, const char *str)
{
	unsigned int b[6] = { 0, 0, 0, 0, 0, 0 };

	if (!mac || !str)
		return -1;
	if (sscanf(str, "%x:%x:%x:%x:%x:%x", &b[0], &b[1], &b[2], &b[3], &b[4], &b[5]) != 6)
		return -1;
	for (int i = 0; i < 6; i++) {
		if (b[i] > 255)
			return -1;
		mac->addr[i] = (uint8_t)b[i];
	}
	return 0;
}
