// mi_cls_kd.hip -- receive delivery on the GPU (mi_cls_deliver_submit).
//
// After a burst is classified, the host decides each frame's fate (parse
// drop, CoS drop / discard, destination pool), takes the packets, and hands
// the device one 48-B mi_cls_dlv_t per delivered packet.  This kernel then
// does the per-packet host steps of loopback_recv / pcapif_recv_pkt that
// follow classification (platform/linux-generic/pktio/loop.c:308-373,
// pcap.c:330-352) straight into page-locked host memory:
//   * the packet's receive metadata (packet_parse_reset + the parse result at
//     the pktio's parser layer, hdr->cos / cls_mark / dst_queue of
//     _odp_cls_classify_packet, odp_classification.c:1742-1771, hdr->input);
//   * the frame copied into the packet's buffer (pcap frames, the pool switch
//     of _odp_pktio_packet_to_pool, include/odp_packet_io_internal.h:352-371);
//   * the stable group-by-queue permutation of the burst: _odp_cls_enq
//     (include/odp_classification_internal.h:208-236) enqueues runs of equal
//     (queue, CoS) in arrival order; grouping every packet of a queue in
//     arrival order gives each queue the same sequence with one enqueue per
//     queue.
// One block of 256 threads serves 16 packets (16 lanes each: lane 0 the
// metadata, all 16 the copy in 16-B pieces, 256 B per round); the last block
// builds the permutation.  HBM is not involved: every byte moves over the
// host link, so the kernel's bound is the link, not the chip.
#include "mi_cls_dev.h"

struct DArgs {
	const uint8_t *base;
	const mi_cls_result_t *res;
	const mi_cls_dlv_t *dlv;
	uint32_t n;
	uint32_t layer;
	uint64_t input;
	uint32_t headroom;
	uint32_t data_from_meta;
	uint32_t *perm;
	uint32_t *gcnt;
};

#define DLV_PER_BLOCK 16
#define DLV_THREADS 256

// apply_layer (odp_pktio.c): what a parser layer below L4 keeps of the full
// parse (odp_parse.c:372-414)
__device__ __forceinline__ void dlv_layer(uint32_t layer, uint32_t &fl, uint32_t &err, uint32_t &l4)
{
	const uint32_t L2F = (1u << 3) | (0x3fu << 6);
	const uint32_t L3F = L2F | (1u << 4) | (0x7fu << 12);
	if (layer >= 3u)   // ODP_PROTO_LAYER_L4 / ALL
		return;
	if (layer == 1u) {   // L2
		fl &= L2F;
		err &= 0x01u;
		l4 = 0xFFFFu;
	} else {             // L3
		fl &= L3F | (1u << 30);
		err &= 0x07u;
	}
}

// The last block: the stable permutation of the entries with qid < 64,
// grouped by qid.  The entries' qids are read once into LDS (every load in
// flight at once: the entries are in host memory), then counted, and each
// entry's place = its group's start + the entries of its group before it:
// per 256-entry chunk a ballot loop over each wave's distinct qids gives the
// rank inside the wave, the other waves' counts the rest.  Bursts of more
// than DLV_GROUP_MAX entries are not grouped (the host leaves qid 0xFF;
// mi_cls_deliver_submit checks it).
#define DLV_GROUP_MAX MI_CLS_DLV_GROUP_MAX
__device__ void dlv_group(const DArgs &a)
{
	__shared__ uint8_t s_q[DLV_GROUP_MAX];
	__shared__ uint32_t s_cnt[MI_CLS_DLV_GROUPS];
	__shared__ uint32_t s_pos[MI_CLS_DLV_GROUPS];
	__shared__ uint32_t s_w[DLV_THREADS / WAVE][MI_CLS_DLV_GROUPS];
	const uint32_t t = threadIdx.x, lane = t & (WAVE - 1), wave = t / WAVE;
	const uint32_t n = a.n < DLV_GROUP_MAX ? a.n : DLV_GROUP_MAX;
	if (t < MI_CLS_DLV_GROUPS)
		s_cnt[t] = 0u;
	{
		// 32 qids per thread, loaded before any is used
		uint8_t q[DLV_GROUP_MAX / DLV_THREADS];
#pragma unroll
		for (uint32_t k = 0; k < DLV_GROUP_MAX / DLV_THREADS; ++k) {
			const uint32_t i = t + k * DLV_THREADS;
			q[k] = i < n ? a.dlv[i].qid : (uint8_t)0xFFu;
		}
#pragma unroll
		for (uint32_t k = 0; k < DLV_GROUP_MAX / DLV_THREADS; ++k)
			s_q[t + k * DLV_THREADS] = q[k];
	}
	__syncthreads();
	for (uint32_t i = t; i < n; i += DLV_THREADS)
		if (s_q[i] < MI_CLS_DLV_GROUPS)
			atomicAdd(&s_cnt[s_q[i]], 1u);
	__syncthreads();
	if (t == 0) {
		uint32_t at = 0;
		for (uint32_t g = 0; g < MI_CLS_DLV_GROUPS; ++g) {
			s_pos[g] = at;
			at += s_cnt[g];
		}
	}
	if (t < MI_CLS_DLV_GROUPS)
		a.gcnt[t] = s_cnt[t];
	__syncthreads();
	const unsigned long long lt = lane ? (~0ull >> (64u - lane)) : 0ull;
	for (uint32_t c0 = 0; c0 < n; c0 += DLV_THREADS) {
		const uint32_t i = c0 + t;
		const uint32_t q = i < n ? s_q[i] : 0xFFu;
		bool left = q < MI_CLS_DLV_GROUPS;
		uint32_t rank = 0;
		for (uint32_t g = lane; g < MI_CLS_DLV_GROUPS; g += WAVE)
			s_w[wave][g] = 0u;
		__syncthreads();
		for (;;) {
			const unsigned long long m = __ballot(left);
			if (!m)
				break;
			const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)q, (int)__builtin_ctzll(m));
			const unsigned long long mv = __ballot(left && q == v);
			if (left && q == v) {
				rank = (uint32_t)__popcll(mv & lt);
				left = false;
			}
			if (lane == 0)
				s_w[wave][v] = (uint32_t)__popcll(mv);
		}
		__syncthreads();
		if (q < MI_CLS_DLV_GROUPS) {
			uint32_t before = 0;
			for (uint32_t w = 0; w < wave; ++w)
				before += s_w[w][q];
			a.perm[s_pos[q] + before + rank] = i;
		}
		__syncthreads();
		if (t < MI_CLS_DLV_GROUPS) {
			uint32_t all = 0;
			for (uint32_t w = 0; w < DLV_THREADS / WAVE; ++w)
				all += s_w[w][t];
			s_pos[t] += all;
		}
		__syncthreads();
	}
}

// One packet's metadata block (64 B, one cache line of its header): four
// 16-B stores by lanes 0-3 of its 16-lane group, so the line crosses the
// host link as one full write (no read-modify-write at the host, and the
// header line the pool and queues use is not touched).
__global__ __launch_bounds__(DLV_THREADS) void mi_cls_deliver_kernel(DArgs a)
{
	if (blockIdx.x == gridDim.x - 1) {
		dlv_group(a);
		return;
	}
	const uint32_t sub = threadIdx.x & 15u;
	const uint32_t j = blockIdx.x * DLV_PER_BLOCK + (threadIdx.x >> 4);
	if (j >= a.n)
		return;
	const mi_cls_dlv_t d = a.dlv[j];
	uint8_t *meta = (uint8_t *)(uintptr_t)d.meta;
	if (sub < 4u) {
		const mi_cls_result_t r = a.res[d.rec];
		uint32_t fl = r.in_flags, err = r.err, l4 = r.l4_offset;
		dlv_layer(a.layer, fl, err, l4);
		const bool cls = (d.flags & MI_CLS_DLV_CLS) != 0u;
		const bool fresh = (d.flags & MI_CLS_DLV_FRESH) != 0u;
		uint32_t cos = 0xFFu, mark = 0u;
		uint64_t dq = 0u;
		if (cls) {
			cos = r.cos;
			mark = r.mark;
			dq = d.dst_queue;
		} else if (!fresh) {
			// parser-only pktio, packet received as it was sent: its
			// classification fields stay
			const mi_cls_pkt_meta_t *m = (const mi_cls_pkt_meta_t *)meta;
			cos = m->cos;
			mark = m->cls_mark;
			dq = m->dst_queue;
		}
		const uint64_t up = fresh ? 0u : d.user_ptr;
		u32x4 v;
		if (sub == 0u) {
			// data_off, len, in_flags (bits 32-63 are never set on this path)
			v = u32x4{ fresh ? a.headroom : d.data_off, d.len, fl, 0u };
		} else if (sub == 1u) {
			// err, cos, cls_mark | l2, l3 | l4, rsv0 | rsv1
			v = u32x4{ err | (cos << 8) | (mark << 16), (uint32_t)r.l3_offset << 16, l4, 0u };
		} else if (sub == 2u) {
			v = u32x4{ (uint32_t)dq, (uint32_t)(dq >> 32), (uint32_t)a.input,
				   (uint32_t)(a.input >> 32) };
		} else {
			v = u32x4{ (uint32_t)up, (uint32_t)(up >> 32), 0u, 0u };
		}
		((u32x4 *)meta)[sub] = v;
	}
	if (d.flags & MI_CLS_DLV_COPY) {
		// the frame in rounds of 1536 B: each lane's six 16-B loads are all
		// issued before its stores (host-memory reads: a latency each)
		const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
			(void *)a.base, (short)0, (int)OOB_OFF, 0x00020000);
		u32x4 *dst = (u32x4 *)(meta + a.data_from_meta);
		for (uint32_t o0 = 16u * sub; o0 < d.len; o0 += 6u * 256u) {
			u32x4 v[6];
#pragma unroll
			for (uint32_t k = 0; k < 6; ++k) {
				const uint32_t o = o0 + 256u * k;
				v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, o < d.len ? d.src + o : OOB_OFF, 0, 0);
			}
#pragma unroll
			for (uint32_t k = 0; k < 6; ++k) {
				const uint32_t o = o0 + 256u * k;
				if (o < d.len)
					dst[o >> 4] = v[k];
			}
		}
	}
}

int mi_cls_launch_deliver(unsigned grid, hipStream_t st, const mi_cls_dlv_args_t &h)
{
	DArgs a;
	a.base = h.base;
	a.res = h.res;
	a.dlv = h.dlv;
	a.n = h.n;
	a.layer = h.layer;
	a.input = h.input;
	a.headroom = h.headroom;
	a.data_from_meta = h.data_from_meta;
	a.perm = h.perm;
	a.gcnt = h.gcnt;
	if (grid == 0) {   // preload (mi_cls_ctx_create)
		hipFuncAttributes fa;
		return hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&mi_cls_deliver_kernel)) ==
		       hipSuccess ? 0 : -EIO;
	}
	void *args[] = { &a };
	return hipLaunchKernel(reinterpret_cast<const void *>(&mi_cls_deliver_kernel), dim3(grid),
			       dim3(DLV_THREADS), args, 0, st) == hipSuccess ? 0 : -EIO;
}

// ------------------------------------------------------------ receive chain
// mi_cls_rx_chain_submit: after the burst's classification, on the device:
// the per-frame decisions the host made for mi_cls_deliver_submit (one
// block: mi_cls_rx_decide_kernel) and the delivery (mi_cls_rx_deliver_kernel).
// The classifier is on, so the parser layer is ALL (odp_packet_io.c:
// 675-677): records need no layer cut.
#define RXD_THREADS 1024
#define RXD_WAVES (RXD_THREADS / WAVE)

// Decisions of frames [0, n) in arrival order: fate, pool slot, the frame's
// rank among its slot's frames (which packet of the slot it takes), queue
// group; the pktio counters; the stable grouping by queue (as dlv_group);
// `short_pool` when a slot has too few packets.  One block of 16 waves.
// Latency rules it, not bytes:
//  - every load of the inputs (records in HBM; lengths, pools and the table
//    in host memory) is issued before any is used, and each thread's frames
//    stay in registers (fully unrolled, constant indexes: nothing in scratch);
//  - the ranks are scans over LDS, one wave per pool slot (16) and per four
//    queue groups (64): a ballot per 64 frames, so 5 barriers per burst, not
//    3 per 1024 frames and a ballot per distinct value;
//  - every store goes out after the last barrier: a barrier waits for the
//    block's outstanding stores, which to host memory take a host-link round
//    trip each.
#define RXD_PER 8   // frames per thread (MI_CLS_DLV_GROUP_MAX / RXD_THREADS)
#define RXD_SEG 8   // 64-frame segments per batch of LDS reads in the scans
static_assert(RXD_PER * RXD_THREADS == MI_CLS_DLV_GROUP_MAX, "one block holds a burst");
static_assert(RXD_WAVES == MI_CLS_RX_POOLS, "one wave per pool slot");
static_assert(RXD_WAVES * 4 == MI_CLS_DLV_GROUPS, "four queue groups per wave");
__global__ __launch_bounds__(RXD_THREADS) void mi_cls_rx_decide_kernel(mi_cls_rxc_args_t a, mi_cls_rxdev_t d)
{
	__shared__ uint8_t s_k[MI_CLS_DLV_GROUP_MAX];        // fresh frame: its slot, else 0xFF
	__shared__ uint8_t s_q[MI_CLS_DLV_GROUP_MAX];        // its queue group, else 0xFF
	__shared__ uint16_t s_rank[MI_CLS_DLV_GROUP_MAX];    // fresh frame: rank in its slot
	__shared__ uint16_t s_perm[MI_CLS_DLV_GROUP_MAX];
	__shared__ uint32_t s_need[MI_CLS_RX_POOLS];
	__shared__ uint32_t s_gcnt[MI_CLS_DLV_GROUPS], s_gpos[MI_CLS_DLV_GROUPS];
	__shared__ uint32_t s_ctr[4];
	__shared__ uint8_t s_cpool[256], s_rts[64], s_qg[MI_CLS_RX_QENT];
	__shared__ uint16_t s_q0[256];
	__shared__ uint64_t s_qh[MI_CLS_RX_QENT];
	__shared__ uint32_t s_cap[MI_CLS_RX_POOLS], s_have[MI_CLS_RX_POOLS];
	const uint32_t t = threadIdx.x, lane = t & (WAVE - 1), wave = t / WAVE;
	const mi_cls_rxtab_t &tab = *d.tab;
	const bool group = (tab.flags & MI_CLS_RXT_GROUP) != 0u;
	const unsigned long long lt = lane ? (~0ull >> (64u - lane)) : 0ull;
	const uint32_t n = a.n, nseg = (n + WAVE - 1u) / WAVE;
	// this thread's frames t, t + 1024, ..: unconditional loads (indexes
	// clamped into the burst, a valid byte array when there is no ppool), so
	// no branch makes the compiler wait for one before the next is issued.
	// The records and the table are in HBM, and so are the lengths and pools
	// of a burst the stage kernel staged: a GPU-staged burst reads nothing
	// over the host link here (reads there queue behind the other burst's
	// delivery traffic)
	mi_cls_result_t r[RXD_PER];
	uint32_t len[RXD_PER], pp[RXD_PER];
	const uint16_t *lena = d.dlen ? d.len : a.slen;
	const uint8_t *ppa = a.pk ? (d.dlen ? d.pp : a.ppool) : (const uint8_t *)lena;
#pragma unroll
	for (uint32_t c = 0; c < RXD_PER; ++c) {
		const uint32_t i = min(c * RXD_THREADS + t, n - 1u);
		r[c] = d.res[i];
		len[c] = lena[i];
		pp[c] = ppa[i];
	}
	// the table's words, also unconditional (wrapped indexes); every thread
	// stores (threads with equal wrapped indexes store the same word): no
	// branch the compiler could sink the loads into
	static_assert(MI_CLS_RX_QENT == RXD_THREADS, "one queue entry per thread");
	{
		const uint8_t cp = tab.cos_pool[t & 255u], qg = tab.qg[t], rs = tab.rt_slot[t & 63u];
		const uint64_t qh = tab.qh[t];
		const uint16_t q0 = tab.cos_q0[t & 255u];
		const uint32_t cap = tab.pool_cap[t & (MI_CLS_RX_POOLS - 1u)];
		const uint32_t hv = a.have[t & (MI_CLS_RX_POOLS - 1u)];
		s_qg[t] = qg;
		s_qh[t] = qh;
		s_cpool[t & 255u] = cp;
		s_q0[t & 255u] = q0;
		s_rts[t & 63u] = rs;
		s_cap[t & (MI_CLS_RX_POOLS - 1u)] = cap;
		s_have[t & (MI_CLS_RX_POOLS - 1u)] = hv;
		s_ctr[t & 3u] = 0u;
	}
	__syncthreads();
	// (1) each frame's fate and slot (odp_packet_io.c:680-705 per frame)
	uint32_t fk[RXD_PER], qe[RXD_PER];
	uint32_t errs = 0, disc = 0;
#pragma unroll
	for (uint32_t c = 0; c < RXD_PER; ++c) {
		const uint32_t i = c * RXD_THREADS + t;
		const bool in = i < n;
		const uint32_t p = a.pk ? pp[c] : 0u;
		uint32_t fate = MI_CLS_RXF_DROP, k = 0u;
		if (in) {
			errs += (r[c].err != 0u || r[c].outcome == MI_CLS_OUT_PARSE_DROP) ? 1u : 0u;
			if (r[c].outcome == MI_CLS_OUT_DISCARD || r[c].outcome == MI_CLS_OUT_LOOP) {
				fate = MI_CLS_RXF_DISCARD;
			} else if (r[c].outcome == MI_CLS_OUT_ENQ) {
				k = s_cpool[r[c].cos] & (MI_CLS_RX_POOLS - 1u);
				const uint32_t own = p ? s_rts[(p - 1u) & 63u] : 0u;
				if (own != 0u && own - 1u == k)
					fate = MI_CLS_RXF_INPLACE;
				else if (len[c] > s_cap[k])
					fate = MI_CLS_RXF_DISCARD;   // odp_packet_alloc fails
				else
					fate = MI_CLS_RXF_FRESH;
			}
			s_k[i] = fate == MI_CLS_RXF_FRESH ? (uint8_t)k : (uint8_t)0xFFu;
		}
		disc += fate == MI_CLS_RXF_DISCARD ? 1u : 0u;
		fk[c] = fate | (k << 2);
		qe[c] = min(in && r[c].outcome == MI_CLS_OUT_ENQ ? s_q0[r[c].cos] + r[c].queue : 0u,
			    (uint32_t)MI_CLS_RX_QENT - 1u);
	}
	__syncthreads();
	// (2) wave k ranks slot k's fresh frames in arrival order (the LDS
	// reads of 8 segments issued together: one read's latency per 8)
	{
		uint32_t base = 0;
		for (uint32_t g0 = 0; g0 < nseg; g0 += RXD_SEG) {
			uint32_t v[RXD_SEG];
#pragma unroll
			for (uint32_t j = 0; j < RXD_SEG; ++j) {
				const uint32_t i = (g0 + j) * WAVE + lane;
				v[j] = i < n ? s_k[i] : 0xFFu;
			}
#pragma unroll
			for (uint32_t j = 0; j < RXD_SEG; ++j) {
				const uint32_t i = (g0 + j) * WAVE + lane;
				const bool mine = v[j] == wave;
				const unsigned long long m = __ballot(mine);
				if (mine)
					s_rank[i] = (uint16_t)min(base + (uint32_t)__popcll(m & lt), 0xFFFFu);
				base += (uint32_t)__popcll(m);
			}
		}
		if (lane == 0)
			s_need[wave] = base;
	}
	__syncthreads();
	// (3) delivered or not, the counters, the queue group
	uint32_t w[RXD_PER];
	uint32_t pkts = 0, octs = 0;
#pragma unroll
	for (uint32_t c = 0; c < RXD_PER; ++c) {
		const uint32_t i = c * RXD_THREADS + t;
		const uint32_t fate = fk[c] & 3u, k = fk[c] >> 2;
		const uint32_t rank = fate == MI_CLS_RXF_FRESH ? s_rank[min(i, n - 1u)] : 0u;
		const bool dlv = (fate == MI_CLS_RXF_FRESH && rank < s_have[k]) || fate == MI_CLS_RXF_INPLACE;
		if (dlv && r[c].err == 0u) {
			++pkts;
			octs += len[c];
		}
		const uint32_t qid = dlv && group ? s_qg[qe[c]] : 0x7Fu;
		w[c] = fk[c] | ((qid & 0x7Fu) << 8) | (rank << 16);
		if (i < n)
			s_q[i] = (uint8_t)(qid < MI_CLS_DLV_GROUPS ? qid : 0xFFu);
	}
	// counters: summed per wave (32-bit: at most 64 x 8 frames of 64 KiB),
	// one LDS add per wave
	{
		uint32_t v[4] = { errs, disc, pkts, octs };
#pragma unroll
		for (int j = 0; j < 4; ++j)
#pragma unroll
			for (int o = 32; o > 0; o >>= 1)
				v[j] += (uint32_t)__shfl_xor((int)v[j], o);
		if (lane == 0) {
#pragma unroll
			for (int j = 0; j < 4; ++j)
				if (v[j])
					atomicAdd(&s_ctr[j], v[j]);
		}
	}
	__syncthreads();
	// (4) the stable permutation of the delivered frames by queue group:
	// wave w counts, then places, groups 4w .. 4w + 3
	uint32_t ngrp = 0;
	if (group) {
		uint32_t cnt[4] = { 0u, 0u, 0u, 0u };
		for (uint32_t g0 = 0; g0 < nseg; g0 += RXD_SEG) {
			uint32_t v[RXD_SEG];
#pragma unroll
			for (uint32_t h = 0; h < RXD_SEG; ++h) {
				const uint32_t i = (g0 + h) * WAVE + lane;
				v[h] = i < n ? s_q[i] : 0xFFu;
			}
#pragma unroll
			for (uint32_t h = 0; h < RXD_SEG; ++h)
#pragma unroll
				for (uint32_t j = 0; j < 4; ++j)
					cnt[j] += (uint32_t)__popcll(__ballot(v[h] == wave * 4u + j));
		}
		if (lane < 4u)
			s_gcnt[wave * 4u + lane] = lane == 0 ? cnt[0] : lane == 1 ? cnt[1] : lane == 2 ? cnt[2] : cnt[3];
		__syncthreads();
		// group starts: every wave sums the counts before its own groups
		uint32_t at[4];
		{
			const uint32_t v = s_gcnt[lane];
			uint32_t below = 0;
			for (uint32_t h = 0; h < MI_CLS_DLV_GROUPS; ++h)
				below += h < wave * 4u ? (uint32_t)__builtin_amdgcn_readlane((int)v, (int)h) : 0u;
			at[0] = below;
			at[1] = at[0] + (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(wave * 4u));
			at[2] = at[1] + (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(wave * 4u + 1u));
			at[3] = at[2] + (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(wave * 4u + 2u));
			for (uint32_t h = 0; h < MI_CLS_DLV_GROUPS; ++h)
				ngrp += (uint32_t)__builtin_amdgcn_readlane((int)v, (int)h);
		}
		for (uint32_t g0 = 0; g0 < nseg; g0 += RXD_SEG) {
			uint32_t v[RXD_SEG];
#pragma unroll
			for (uint32_t h = 0; h < RXD_SEG; ++h) {
				const uint32_t i = (g0 + h) * WAVE + lane;
				v[h] = i < n ? s_q[i] : 0xFFu;
			}
#pragma unroll
			for (uint32_t h = 0; h < RXD_SEG; ++h)
#pragma unroll
				for (uint32_t j = 0; j < 4; ++j) {
					const bool mine = v[h] == wave * 4u + j;
					const unsigned long long m = __ballot(mine);
					if (mine)
						s_perm[at[j] + (uint32_t)__popcll(m & lt)] =
							(uint16_t)((g0 + h) * WAVE + lane);
					at[j] += (uint32_t)__popcll(m);
				}
		}
		__syncthreads();
	}
	// every output, after the last barrier
#pragma unroll
	for (uint32_t c = 0; c < RXD_PER; ++c) {
		const uint32_t i = c * RXD_THREADS + t;
		if (i >= n)
			continue;
		a.dec[i] = w[c];
		d.dec[i] = w[c];
		d.dq[i] = s_qh[qe[c]];
	}
	for (uint32_t j = t; j < ngrp; j += RXD_THREADS)
		a.perm[j] = s_perm[j];
	if (group && t < MI_CLS_DLV_GROUPS)
		a.gcnt[t] = s_gcnt[t];
	if (t == 0) {
		a.out->in_errors = s_ctr[0];
		a.out->in_discards = s_ctr[1];
		a.out->packets = s_ctr[2];
		a.out->octets = s_ctr[3];
		uint32_t sh = 0;
		for (uint32_t k = 0; k < MI_CLS_RX_POOLS; ++k) {
			a.out->used[k] = min(s_need[k], s_have[k]);
			a.out->need[k] = s_need[k];
			sh |= s_need[k] > s_have[k] ? 1u : 0u;
		}
		a.out->short_pool = sh;
	}
}

// The delivery of the decided frames: 16 frames per block, 16 lanes each
// (lanes 0-3: the 64-B metadata line, all 16: the frame copy), as
// mi_cls_deliver_kernel.  A fresh packet gets the whole line; a loop packet
// received in its own buffer keeps its headroom and user pointer (read from
// its line), and a pool switch takes the old packet's user pointer.
__global__ __launch_bounds__(DLV_THREADS) void mi_cls_rx_deliver_kernel(mi_cls_rxc_args_t a, mi_cls_rxdev_t d)
{
	const uint32_t sub = threadIdx.x & 15u;
	const uint32_t i = blockIdx.x * DLV_PER_BLOCK + (threadIdx.x >> 4);
	if (i >= a.n)
		return;
	// the frame's packet: the rank-th packet taken of its slot, or its own
	const uint32_t dw = d.dec[i], fate = dw & 3u, k = (dw >> 2) & 31u, rank = dw >> 16;
	const bool fresh = fate == MI_CLS_RXF_FRESH;
	const uint64_t e = fresh ? (rank < a.have[k] ? a.got[a.got_base[k] + rank] : 0ull)
				 : (fate == MI_CLS_RXF_INPLACE ? a.pk[i] : 0ull);
	if (sub == 15u)
		a.ent[i] = e;
	if (sub == 14u)
		a.res[i] = d.res[i];   // every frame's record, for the host
	if (!e)
		return;
	uint8_t *meta = (uint8_t *)(uintptr_t)(e + a.meta_off);
	const uint32_t len = d.dlen ? d.len[i] : a.slen[i];
	if (sub < 4u) {
		const mi_cls_result_t r = d.res[i];
		const uint64_t dq = d.dq[i];
		u32x4 v;
		if (sub == 0u) {
			const uint32_t doff = fresh ? a.headroom : ((const u32x4 *)meta)[0][0];
			v = u32x4{ doff, len, r.in_flags, 0u };
		} else if (sub == 1u) {
			v = u32x4{ (uint32_t)r.err | ((uint32_t)r.cos << 8) | ((uint32_t)r.mark << 16),
				   (uint32_t)r.l3_offset << 16, r.l4_offset, 0u };
		} else if (sub == 2u) {
			v = u32x4{ (uint32_t)dq, (uint32_t)(dq >> 32), (uint32_t)a.input,
				   (uint32_t)(a.input >> 32) };
		} else {
			// user pointer: kept in place; a pool switch takes the old
			// packet's; a pcap frame has none
			uint64_t up = 0u;
			if (!fresh)
				up = ((const mi_cls_pkt_meta_t *)meta)->user_ptr;
			else if (a.pk)
				up = ((const mi_cls_pkt_meta_t *)(uintptr_t)(a.pk[i] + a.meta_off))->user_ptr;
			v = u32x4{ (uint32_t)up, (uint32_t)(up >> 32), 0u, 0u };
		}
		((u32x4 *)meta)[sub] = v;
	}
	if (fresh) {
		const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
			(void *)a.base, (short)0, (int)OOB_OFF, 0x00020000);
		const uint32_t src = a.soff[i];
		u32x4 *dst = (u32x4 *)(meta + a.data_from_meta);
		for (uint32_t o0 = 16u * sub; o0 < len; o0 += 6u * 256u) {
			u32x4 v[6];
#pragma unroll
			for (uint32_t k = 0; k < 6; ++k) {
				const uint32_t o = o0 + 256u * k;
				v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, o < len ? src + o : OOB_OFF, 0, 0);
			}
#pragma unroll
			for (uint32_t k = 0; k < 6; ++k) {
				const uint32_t o = o0 + 256u * k;
				if (o < len)
					dst[o >> 4] = v[k];
			}
		}
	}
}

// Loop receive staging on the device (args.stage): each frame's descriptor
// from its packet's header -- the data address (buffer + headroom) relative
// to the burst's base, the length, the pool -- as the host's stage_frames
// builds it for packets in page-locked pools.  A packet outside the
// page-locked range gets an empty descriptor and sets not_in_place (the
// host then stages and delivers the burst itself).
__global__ __launch_bounds__(256) void mi_cls_rx_stage_kernel(mi_cls_rxc_args_t a, mi_cls_rxdev_t d, uint64_t bytes)
{
	// the page-locked flags go to LDS while the handles load (two host-link
	// round trips per frame: the handle, then its header's words)
	__shared__ uint8_t s_pin[64];
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	const uint8_t pin = d.tab->rt_pinned[threadIdx.x & 63u];
	const uint64_t hp = a.pk[min(i, a.n - 1u)];
	s_pin[threadIdx.x & 63u] = pin;
	__syncthreads();
	if (i >= a.n)
		return;
	const uint8_t *h = (const uint8_t *)(uintptr_t)hp;
	const uint64_t head = *(const uint64_t *)(h + a.head_off);
	const uint32_t pool = *(const uint16_t *)(h + a.pool_off);
	const mi_cls_pkt_meta_t *m = (const mi_cls_pkt_meta_t *)(h + a.meta_off);
	const uint64_t da = head + m->data_off, base = (uint64_t)(uintptr_t)a.base;
	const uint32_t l = min(m->len, 65535u);
	const bool ok = pool < 64u && s_pin[pool] && da >= base && da - base + l + 16u <= bytes;
	((uint32_t *)a.soff)[i] = ok ? (uint32_t)(da - base) : 0u;
	((uint16_t *)a.slen)[i] = ok ? (uint16_t)l : (uint16_t)0;
	((uint8_t *)a.ppool)[i] = (uint8_t)(pool + 1u);
	d.len[i] = ok ? (uint16_t)l : (uint16_t)0;
	d.pp[i] = (uint8_t)(pool + 1u);
	if (!ok)
		a.out->not_in_place = 1u;
}

int mi_cls_launch_rx_stage(hipStream_t st, const mi_cls_rxc_args_t &a, const mi_cls_rxdev_t &d, uint64_t bytes,
			   bool preload)
{
	if (preload) {
		hipFuncAttributes fa;
		return hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&mi_cls_rx_stage_kernel)) ==
		       hipSuccess ? 0 : -EIO;
	}
	mi_cls_rxc_args_t h = a;
	mi_cls_rxdev_t hd = d;
	uint64_t b = bytes;
	void *args[] = { &h, &hd, &b };
	return hipLaunchKernel(reinterpret_cast<const void *>(&mi_cls_rx_stage_kernel),
			       dim3((a.n + 255u) / 256u), dim3(256), args, 0, st) == hipSuccess ? 0 : -EIO;
}

int mi_cls_launch_rx_chain(hipStream_t st, const mi_cls_rxc_args_t &a, const mi_cls_rxdev_t &d, bool preload)
{
	if (preload) {
		hipFuncAttributes fa;
		return hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&mi_cls_rx_decide_kernel)) ==
				       hipSuccess &&
			       hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&mi_cls_rx_deliver_kernel)) ==
				       hipSuccess ? 0 : -EIO;
	}
	mi_cls_rxc_args_t h = a;
	mi_cls_rxdev_t hd = d;
	void *args[] = { &h, &hd };
	if (hipLaunchKernel(reinterpret_cast<const void *>(&mi_cls_rx_decide_kernel), dim3(1),
			    dim3(RXD_THREADS), args, 0, st) != hipSuccess)
		return -EIO;
	const unsigned grid = (a.n + DLV_PER_BLOCK - 1u) / DLV_PER_BLOCK;
	return hipLaunchKernel(reinterpret_cast<const void *>(&mi_cls_rx_deliver_kernel), dim3(grid),
			       dim3(DLV_THREADS), args, 0, st) == hipSuccess ? 0 : -EIO;
}
