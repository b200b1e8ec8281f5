// mi_cls.hip -- host side of the MI355X packet parse + PMR classify path: the
// C ABI declared in include/mi_cls.h (contexts, rule-table assembly into the
// device encoding, launches, host-batch staging, statistics).  The kernel
// itself is in mi_cls_dev.h, instantiated per block shape in
// mi_cls_k4/8/12/16.hip.
#include "mi_cls_dev.h"

#include <thread>

// ------------------------------------------------------------------- host
struct mi_cls_ctx {
	int device;
	uint32_t *d_dev;         // assembled device rule program
	size_t dev_cap;          // bytes
	int loaded;
	uint32_t hot_words;      // size of the program's hot region
	int tree;                // some rule leads to a CoS with rules (DIV kernel)
	int flat_mode;           // engine of the default CoS block when every packet is
	                         // decided there in one round (flat kernels), else -1
	int wpb;                 // forced waves per block (MI_CLS_WPB at load), 0 = auto
	uint32_t opt;            // pktin options (mi_cls_pktin_opt_set)
	unsigned long long *d_stats;
	uint32_t *d_hint;        // window hint word (KArgs.hint)
	uint32_t seq;            // launches so far
	int stats_on;
	uint32_t stats_mask[8];
	int num_cu;
	// host-batch staging (mi_cls_classify_host)
	hipStream_t stream;
	uint32_t *h_off;         // pinned: rebased descriptors of a slice
	mi_cls_result_t *h_out;  // pinned: records of a slice (multi-GPU)
	uint8_t *d_pk;
	size_t pk_cap;
	uint32_t *d_off;
	uint16_t *d_len;
	mi_cls_result_t *d_out;
	uint32_t n_cap;
	// submitted host batches (mi_cls_classify_host_submit): completion
	// events in a ring, tickets numbered from 1
	hipEvent_t ev[8];
	uint64_t submitted;
};

#define HIP_OK(x) do { if ((x) != hipSuccess) return -EIO; } while (0)

extern "C" int mi_cls_device_count(void)
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess)
		return 0;
	return n;
}

extern "C" int mi_cls_ctx_create(int device, mi_cls_ctx_t **out)
{
	if (!out)
		return -EINVAL;
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
		return -ENODEV;
	mi_cls_ctx_t *c = (mi_cls_ctx_t *)calloc(1, sizeof(*c));
	if (!c)
		return -ENOMEM;
	c->device = device;
	int cur = 0;
	(void)hipGetDevice(&cur);
	if (hipSetDevice(device) != hipSuccess) {
		free(c);
		return -EIO;
	}
	hipDeviceProp_t prop;
	if (hipGetDeviceProperties(&prop, device) == hipSuccess)
		c->num_cu = prop.multiProcessorCount;
	else
		c->num_cu = 256;
	if (hipMalloc((void **)&c->d_stats, MAX_STATS_COS * sizeof(unsigned long long)) != hipSuccess ||
	    hipMemset(c->d_stats, 0, MAX_STATS_COS * sizeof(unsigned long long)) != hipSuccess ||
	    hipMalloc((void **)&c->d_hint, sizeof(uint32_t)) != hipSuccess ||
	    hipMemset(c->d_hint, 0, sizeof(uint32_t)) != hipSuccess) {
		free(c);
		(void)hipSetDevice(cur);
		return -ENOMEM;
	}
	(void)hipSetDevice(cur);
	*out = c;
	return 0;
}

extern "C" int mi_cls_ctx_destroy(mi_cls_ctx_t *c)
{
	if (!c)
		return -EINVAL;
	(void)hipSetDevice(c->device);
	if (c->d_dev)
		(void)hipFree(c->d_dev);
	if (c->d_stats)
		(void)hipFree(c->d_stats);
	if (c->d_hint)
		(void)hipFree(c->d_hint);
	if (c->stream) {
		(void)hipStreamSynchronize(c->stream);
		(void)hipStreamDestroy(c->stream);
	}
	for (int i = 0; i < 8; ++i)
		if (c->ev[i])
			(void)hipEventDestroy(c->ev[i]);
	(void)hipFree(c->d_pk);
	(void)hipFree(c->d_off);
	(void)hipFree(c->d_len);
	(void)hipFree(c->d_out);
	(void)hipHostFree(c->h_off);
	(void)hipHostFree(c->h_out);
	free(c);
	return 0;
}

static int validate_tbl(const void *tbl, size_t bytes)
{
	if (!tbl || bytes < sizeof(mi_tbl_hdr_t))
		return -EINVAL;
	const mi_tbl_hdr_t *h = (const mi_tbl_hdr_t *)tbl;
	if (h->magic != MI_CLS_TBL_MAGIC || h->version != MI_CLS_TBL_VERSION || h->total_bytes != bytes)
		return -EINVAL;
	if (h->num_cos > 256 || h->cos_off != sizeof(mi_tbl_hdr_t))
		return -EINVAL;
	if ((uint64_t)h->rule_off != (uint64_t)h->cos_off + (uint64_t)h->num_cos * sizeof(mi_cos_t) ||
	    (uint64_t)h->term_off != (uint64_t)h->rule_off + (uint64_t)h->num_rules * sizeof(mi_rule_t) ||
	    (uint64_t)h->total_bytes != (uint64_t)h->term_off + (uint64_t)h->num_terms * sizeof(mi_term_t))
		return -EINVAL;
	if (h->default_cos >= (int32_t)h->num_cos || h->error_cos >= (int32_t)h->num_cos ||
	    h->default_cos < -1 || h->error_cos < -1)
		return -EINVAL;
	// every index the kernel follows must stay inside the table
	const uint8_t *b = (const uint8_t *)tbl;
	const mi_cos_t *cs = (const mi_cos_t *)(b + h->cos_off);
	const mi_rule_t *rs = (const mi_rule_t *)(b + h->rule_off);
	const mi_term_t *ts = (const mi_term_t *)(b + h->term_off);
	for (uint32_t i = 0; i < h->num_cos; ++i) {
		if ((uint64_t)cs[i].rule_begin + cs[i].num_rules > h->num_rules)
			return -EINVAL;
		if (cs[i].num_queue < 1 || cs[i].num_queue > 32)
			return -EINVAL;
	}
	for (uint32_t i = 0; i < h->num_rules; ++i) {
		if (rs[i].dst_cos >= h->num_cos || rs[i].num_terms > 8 ||
		    (uint64_t)rs[i].term_begin + rs[i].num_terms > h->num_terms)
			return -EINVAL;
	}
	for (uint32_t i = 0; i < h->num_terms; ++i) {
		if (ts[i].kind >= MI_K_COUNT || ts[i].size > 16)
			return -EINVAL;
	}
	return 0;
}

// Mask word i of a term as the kernel applies it: the term's mask cut down
// to the field's own bits in the 4-byte word the kernel reads (the kernel
// reads every fixed field as a whole little-endian word, see fdesc()).
static uint32_t eff_mask(const mi_term_t &t, uint32_t i)
{
	switch (t.kind) {
	case MI_K_ETH0:
	case MI_K_ETHX:
		return t.mask[i] & 0xffffu;
	case MI_K_VID0:
	case MI_K_VIDX:
		return t.mask[i] & 0xff0fu;      // VLAN ID bits of the raw TCI
	case MI_K_PROTO:
		return t.mask[i] & 0xffu;
	case MI_K_DMAC:
		return i == 1 ? (t.mask[i] & 0xffffu) : t.mask[i];
	default:
		return t.mask[i];
	}
}

// words of one term in the device encoding (see "device rule program")
static uint32_t encode_term(const mi_term_t &t, uint32_t *w)
{
	uint32_t n = 0;
	if (t.kind == MI_K_CUSTOM_FRAME || t.kind == MI_K_CUSTOM_L3) {
		uint32_t nw = (t.size + 3u) / 4u;
		w[n++] = t.kind | ((uint32_t)t.size << 8) | (nw << 16);
		w[n++] = t.offset;
		for (uint32_t i = 0; i < nw; ++i) {
			w[n++] = t.mask[i];
			w[n++] = t.value[i];
		}
		return n;
	}
	uint32_t nw = (t.kind == MI_K_SIP6 || t.kind == MI_K_DIP6) ? 4u : (t.kind == MI_K_DMAC ? 2u : 1u);
	w[n++] = t.kind | ((uint32_t)t.size << 8) | (nw << 16);
	for (uint32_t i = 0; i < nw; ++i) {
		w[n++] = eff_mask(t, i);
		w[n++] = t.value[i];
	}
	return n;
}

// key words a term kind reads (encode_term's nw)
static uint32_t kind_words(uint32_t kind, uint32_t size)
{
	if (kind == MI_K_CUSTOM_FRAME || kind == MI_K_CUSTOM_L3)
		return (size + 3u) / 4u;
	return (kind == MI_K_SIP6 || kind == MI_K_DIP6) ? 4u : (kind == MI_K_DMAC ? 2u : 1u);
}

// ---- bit-vector block construction (host) ----
struct ClassKey {
	uint32_t kind, nkey, offset, size, mask[4];
	bool operator<(const ClassKey &o) const
	{
		if (kind != o.kind) return kind < o.kind;
		if (offset != o.offset) return offset < o.offset;
		if (size != o.size) return size < o.size;
		for (int i = 0; i < 4; ++i)
			if (mask[i] != o.mask[i]) return mask[i] < o.mask[i];
		return false;
	}
};

typedef std::array<uint32_t, 4> Key4;

// fold of a key's words (same as bv_fold on the device)
static uint32_t host_bv_fold(const Key4 &k)
{
	// keep in step with bv_fold()
	uint32_t h = k[0] * 0x9E3779B1u ^ k[1] * 0x85EBCA77u ^ k[2] * 0xC2B2AE3Du ^ k[3] * 0x27D4EB2Fu;
	return h ^ (h >> 15);
}

// bv_bucket() on the host: x = key word or fold, nb buckets
static uint32_t host_bucket(uint32_t x, uint32_t mult, uint32_t nb)
{
	const uint32_t y = (x ^ (x >> 16)) & 0xFFFFFFu;
	const uint32_t h = (uint32_t)(y * (uint64_t)(mult & 0xFFFFFFu));
	return (uint32_t)(((uint64_t)(h >> 16) * nb) >> 16);
}

// Two-choice cuckoo table over `keys`: every key sits in a slot of bucket
// b1 or b2 (a lookup reads both buckets at once, no probe loop).  bsz slots
// per bucket: 2 for one-word keys (a 16-B bucket, load <= 87.5 %), 1 for
// longer keys (load <= 45 %).  Returns the slot (bucket * bsz + j) of every
// key, the bucket count and the multipliers used.
static bool cuckoo_place(const std::vector<Key4> &keys, uint32_t nk, uint32_t bsz, uint32_t &nb_out,
			 uint32_t &m1, uint32_t &m2, std::vector<uint32_t> &slot_of)
{
	const uint32_t n = (uint32_t)keys.size();
	std::vector<uint32_t> fold(n);
	for (uint32_t i = 0; i < n; ++i)
		fold[i] = nk == 1 ? keys[i][0] : host_bv_fold(keys[i]);
	// load <= 87.5 % with 2-slot buckets (below the ~89.7 % two-choice
	// threshold; a failed placement grows the table), <= 45 % otherwise
	uint32_t nb = bsz == 2 ? (n * 4 + 6) / 7 : (n * 20 + 8) / 9 + 1;
	if (nb < 1)
		nb = 1;
	uint64_t rng = 0x9E3779B97F4A7C15ull ^ ((uint64_t)n << 17);
	for (int grow = 0; grow < 8 && nb <= 65536u; ++grow, nb += nb / 8 + 1) {
		nb_out = nb;
		for (int attempt = 0; attempt < 64; ++attempt) {
			rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
			m1 = ((uint32_t)rng & 0xFFFFFFu) | 1u;
			rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
			m2 = ((uint32_t)(rng >> 32) & 0xFFFFFFu) | 1u;
			std::vector<int32_t> occ((size_t)nb * bsz, -1);
			slot_of.assign(n, 0);
			bool ok = true;
			for (uint32_t i = 0; i < n && ok; ++i) {
				uint32_t cur = i, b = host_bucket(fold[i], m1, nb);
				for (int kick = 0;; ++kick) {
					// a free slot in either bucket of `cur`
					const uint32_t c1 = host_bucket(fold[cur], m1, nb);
					const uint32_t c2 = host_bucket(fold[cur], m2, nb);
					int32_t fs = -1;
					for (uint32_t bb : { c1, c2 })
						for (uint32_t j = 0; j < bsz && fs < 0; ++j)
							if (occ[(size_t)bb * bsz + j] < 0)
								fs = (int32_t)(bb * bsz + j);
					if (fs >= 0) {
						occ[fs] = (int32_t)cur;
						slot_of[cur] = (uint32_t)fs;
						break;
					}
					if (kick > 500) {
						ok = false;
						break;
					}
					// evict a pseudo-random slot of bucket b (alternating buckets)
					rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
					const uint32_t sl = b * bsz + (uint32_t)(rng % bsz);
					const uint32_t ev = (uint32_t)occ[sl];
					occ[sl] = (int32_t)cur;
					slot_of[cur] = sl;
					cur = ev;
					const uint32_t e1 = host_bucket(fold[ev], m1, nb);
					const uint32_t e2 = host_bucket(fold[ev], m2, nb);
					b = e1 == b ? e2 : e1;
				}
			}
			if (ok) {
				// every key must sit in one of its two buckets
				for (uint32_t i = 0; i < n && ok; ++i) {
					const uint32_t bk = slot_of[i] / bsz;
					ok = occ[slot_of[i]] == (int32_t)i &&
					     (bk == host_bucket(fold[i], m1, nb) ||
					      bk == host_bucket(fold[i], m2, nb));
				}
				if (ok)
					return true;
				fprintf(stderr, "mi_cls: cuckoo placement self-check failed\n");
			}
		}
	}
	return false;
}

static bool class_of(const mi_term_t &t, ClassKey &ck)
{
	memset(&ck, 0, sizeof(ck));
	ck.kind = t.kind;
	switch (t.kind) {
	case MI_K_NEVER:
	case MI_K_ALWAYS:
		return false;
	case MI_K_CUSTOM_FRAME:
	case MI_K_CUSTOM_L3:
		ck.offset = t.offset;
		ck.size = t.size;
		ck.nkey = t.size > 8 ? 4 : (t.size > 4 ? 2 : 1);
		break;
	case MI_K_SIP6:
	case MI_K_DIP6:
		ck.nkey = 4;
		break;
	case MI_K_DMAC:
		ck.nkey = 2;
		break;
	default:
		ck.nkey = 1;
	}
	for (uint32_t i = 0; i < 4; ++i)
		ck.mask[i] = i < ck.nkey ? eff_mask(t, i) : 0;
	// trailing key words the mask clears are not part of the key (an IPv6
	// /64 prefix is a two-word key: half the key reads, 16-B table slots)
	while (ck.nkey > 1 && ck.mask[ck.nkey - 1] == 0)
		--ck.nkey;
	// UDP and TCP port terms read the same bytes (the raw port word at l4)
	// under different gates: one class for both, the protocol carried in
	// two key bits the mask leaves free (tag 1 UDP, 2 TCP; port masks are
	// <= 16 bits, so bits tp, tp+1 exist), so a packet's key holds its
	// protocol and one lookup serves rules of either kind.
	static const bool no_merge = getenv("MI_CLS_NO_PORTMERGE") != nullptr;   // A/B, tests
	if (!no_merge && (t.kind == MI_K_UDP_DPORT || t.kind == MI_K_TCP_DPORT ||
			  t.kind == MI_K_UDP_SPORT || t.kind == MI_K_TCP_SPORT)) {
		uint32_t tp = 0;
		while (tp < 31 && ((ck.mask[0] >> tp) & 3u))
			++tp;
		if (tp < 31) {
			ck.kind = K_L4PORT;
			ck.offset = tp;
		}
	}
	return true;
}

// value words a term requires of its class (the tag of a merged port class)
static Key4 class_value(const mi_term_t &t, const ClassKey &ck)
{
	Key4 v = { 0, 0, 0, 0 };
	for (uint32_t i = 0; i < ck.nkey; ++i)
		v[i] = t.value[i];
	if (ck.kind == K_L4PORT)
		v[0] |= (t.kind == MI_K_UDP_DPORT || t.kind == MI_K_UDP_SPORT ? 1u : 2u) << ck.offset;
	return v;
}

// Build the classification block of one CoS into `blk` (word offsets are
// relative to the start of the hot region; base = blk's first word index).
// Returns false when the CoS needs more than BV_MAX_CLS key classes or its
// candidate lists degenerate (the linear scan is used instead).
//
// Semantics (match_pmr_cos, odp_classification.c:1624-1667): the CoS's
// result is the FIRST rule in scan order all of whose terms hold.  A rule's
// terms are grouped by key class (term kind + mask [+ offset, size]); a rule
// holds iff for every class it constrains the packet has the field and the
// masked field equals the rule's value (two terms of one class with
// different values, or an LD_VNI term, make it unmatchable -- not "alive").
// Every class has a cuckoo table keyed by the values its rules require; a
// packet's lookup (absent field = miss) selects:
//  * DIRECT mode (one class): the first alive rule among "rules with this
//    key or without a term of the class" (stored as 1 + rule); a miss takes
//    the first alive rule without a term of the class.
//  * BITMAP mode (<= 32 rules): the 32-bit row "rules with this key or
//    without a term of the class"; a miss takes the row of the latter.  The
//    AND of the rows with the alive row has the first holding rule as its
//    lowest set bit.
//  * CANDIDATE mode: every distinct (class, value) has a key id (1..); the
//    lookup gives the packet's key id (0: miss).  Every constraining rule is
//    filed under ONE of its classes -- its "primary", the one whose value
//    the fewest rules share -- in a list per key id in scan order.  The
//    candidates are the lists of the packet's key ids plus the first rule
//    with no classified term (it matches everything); a candidate holds iff
//    its record's key ids equal the packet's, and the smallest one wins.
static bool build_bv(const mi_cos_t *cs, const mi_rule_t *rs, const mi_term_t *ts, uint32_t nrules,
		     uint32_t base, std::vector<uint32_t> &blk,
		     std::vector<std::pair<uint32_t, std::array<uint32_t, 16>>> &shared)
{
	std::map<ClassKey, uint32_t> cls;
	std::vector<ClassKey> cls_list;
	for (uint32_t r = 0; r < nrules; ++r)
		for (uint32_t t = 0; t < rs[r].num_terms; ++t) {
			ClassKey ck;
			if (class_of(ts[rs[r].term_begin + t], ck) && !cls.count(ck)) {
				cls[ck] = (uint32_t)cls_list.size();
				cls_list.push_back(ck);
			}
		}
	const uint32_t ncls = (uint32_t)cls_list.size();
	if (ncls > BV_MAX_CLS || ncls == 0)
		return false;
	// canonical class order: CoS with the same classes evaluate them in the
	// same order, so lanes on different CoS stay convergent
	std::sort(cls_list.begin(), cls_list.end());
	for (uint32_t i = 0; i < ncls; ++i)
		cls[cls_list[i]] = i;
	// per rule: alive, constrained classes and their values
	std::vector<uint8_t> alive(nrules, 0);
	std::vector<uint32_t> tmask(nrules, 0);
	std::vector<std::vector<Key4>> want(nrules, std::vector<Key4>(ncls));
	std::vector<std::map<Key4, uint32_t>> freq(ncls);   // value -> #alive rules
	for (uint32_t r = 0; r < nrules; ++r) {
		bool ok = true;
		for (uint32_t t = 0; t < rs[r].num_terms; ++t) {
			const mi_term_t &tm = ts[rs[r].term_begin + t];
			ClassKey ck;
			if (!class_of(tm, ck)) {
				if (tm.kind == MI_K_NEVER)
					ok = false;
				continue;
			}
			const uint32_t c = cls[ck];
			const Key4 v = class_value(tm, ck);
			// a value bit under a zero mask word (trimmed from the key) can
			// never be matched; values are pre-masked by the control plane,
			// this guards other producers of the table
			for (uint32_t i = ck.nkey; i < 4; ++i)
				if ((kind_words(tm.kind, tm.size) > i) && tm.value[i] != 0u)
					ok = false;
			if (((tmask[r] >> c) & 1u) && want[r][c] != v)
				ok = false;   // two terms of one class with different values
			tmask[r] |= 1u << c;
			want[r][c] = v;
		}
		if (!ok)
			continue;
		alive[r] = 1;
		for (uint32_t c = 0; c < ncls; ++c)
			if ((tmask[r] >> c) & 1u)
				freq[c][want[r][c]]++;
	}
	// primary class of every alive constrained rule: the class whose value
	// the fewest alive rules share (candidate engines file the rule under it)
	std::vector<uint32_t> prim_of(nrules, BV_NONE);
	std::vector<std::map<Key4, uint32_t>> filed(ncls);   // value -> #rules filed
	uint32_t max_list = 0, prim_mask = 0;
	for (uint32_t r = 0; r < nrules; ++r) {
		if (!alive[r] || tmask[r] == 0u)
			continue;
		uint32_t best = 0xFFFFFFFFu;
		for (uint32_t c = 0; c < ncls; ++c)
			if (((tmask[r] >> c) & 1u) && freq[c][want[r][c]] < best) {
				best = freq[c][want[r][c]];
				prim_of[r] = c;
			}
		const uint32_t c = prim_of[r];
		max_list = std::max(max_list, ++filed[c][want[r][c]]);
		prim_mask |= 1u << c;
	}
	// MI_CLS_NO_WIDE: candidate lists instead of wide rows; MI_CLS_NO_CAND1:
	// no single-candidate engine (A/B, tests)
	const bool wide_ok = getenv("MI_CLS_NO_WIDE") == nullptr;
	const bool cand1_ok = getenv("MI_CLS_NO_CAND1") == nullptr;
	const uint32_t mode = ncls == 1 ? 0u
		: (nrules <= 32 ? 2u
		: ((cand1_ok && max_list <= 1u && nrules < 0xFFFFu) ? 4u
		: ((wide_ok && nrules <= 32 * BV_WIDE_WORDS) ? 3u : 1u)));
	std::vector<std::map<Key4, uint32_t>> kid(ncls);   // value -> key id (1..)
	for (uint32_t c = 0; c < ncls; ++c) {
		uint32_t id = 1;
		for (auto &kv : freq[c])
			kid[c][kv.first] = id++;
		if (id > 4096u)
			return false;
	}
	auto holds_class = [&](uint32_t r, uint32_t c, const Key4 *v) {
		return !((tmask[r] >> c) & 1u) || (v && want[r][c] == *v);
	};
	uint32_t wc_first = BV_NONE;   // first alive rule without a classified term
	for (uint32_t r = 0; r < nrules && wc_first == BV_NONE; ++r)
		if (alive[r] && tmask[r] == 0u)
			wc_first = r;
	// header (8) | classes (16 each) | results | [records] | per class: table [, lists].
	// Split class (direct blocks): the 16-word class record holds only what
	// the class is (kind, key words, masks, field descriptor); it is stored
	// once per distinct record in the hot region by assemble(), which
	// patches its index into the block's 6-word class info in header words
	// 2-7 (shared record, miss word, bucket count, table, m1, m2); the block
	// is header | table.  (Splitting the bitmap blocks' classes the same way
	// measured slower on config5: the per-lane rounds read more words.)
	const bool split = mode == 0u;
	blk.assign(mode == 0u ? 8u : 8u + BV_CLS_WORDS * ncls, 0);
	shared.clear();
	blk[0] = mode;
	blk[1] = ncls;
	blk[3] = wc_first;
	auto res_word = [&](uint32_t r) {
		return (rs[r].dst_cos & 0xffu) | (cs[rs[r].dst_cos].num_rules == 0 ? 0x100u : 0u) |
		       ((uint32_t)rs[r].mark << 16);
	};
	// direct blocks keep each rule's result word in the table slot itself
	// (no results array, no second lookup); the others index this array
	blk[2] = base + (uint32_t)blk.size();
	if (mode != 0u)
		for (uint32_t r = 0; r < nrules; ++r)
			blk.push_back(res_word(r));
	std::vector<std::vector<std::vector<uint32_t>>> lists(ncls);   // [class][key id] -> rules
	// wide rows: 8 words each (zero past the rule count), deduplicated.  Every
	// row id is assigned before the layout is emitted (mode 3 below): rows
	// are stored as two arrays of 4-word halves, so a row's value is the
	// hot-region word index of its first half and the second half is
	// blk[7] words further (16-B aligned; consecutive rows 16 B apart)
	const uint32_t nw = (nrules + 31u) / 32u;
	auto wide_row = [&](uint32_t c, const Key4 *v) {
		std::vector<uint32_t> w(BV_WIDE_WORDS, 0u);
		for (uint32_t r = 0; r < nrules; ++r)
			if (holds_class(r, c, v))
				w[r / 32u] |= 1u << (r % 32u);
		return w;
	};
	std::map<std::vector<uint32_t>, uint32_t> row_id;
	std::vector<const std::vector<uint32_t> *> rows;
	auto get_row = [&](const std::vector<uint32_t> &row) -> uint32_t {
		auto it = row_id.find(row);
		if (it != row_id.end())
			return it->second;
		const uint32_t id = (uint32_t)rows.size();
		auto ins = row_id.emplace(row, id).first;
		rows.push_back(&ins->first);
		return id;
	};
	std::vector<uint32_t> miss_id(ncls, 0);
	std::vector<std::vector<uint32_t>> key_row(ncls);
	uint32_t rows_at = 0;   // block-relative index of the first-halves array
	auto align4 = [&]() { while (blk.size() & 3u) blk.push_back(0); };
	if (mode == 2u) {
		uint32_t aw = 0;
		for (uint32_t r = 0; r < nrules; ++r)
			aw |= (uint32_t)alive[r] << r;
		blk[4] = aw;
	} else if (mode == 3u) {
		blk[6] = nw;
		blk[4] = (uint32_t)blk.size();   // the alive row, block-relative
		for (uint32_t i = 0; i < BV_WIDE_WORDS; ++i) {
			uint32_t aw = 0;
			for (uint32_t j = 0; j < 32u && 32u * i + j < nrules; ++j)
				aw |= (uint32_t)alive[32u * i + j] << j;
			blk.push_back(aw);
		}
		for (uint32_t c = 0; c < ncls; ++c) {
			miss_id[c] = get_row(wide_row(c, nullptr));
			for (auto &kv : kid[c])
				key_row[c].push_back(get_row(wide_row(c, &kv.first)));
		}
		align4();
		rows_at = (uint32_t)blk.size();
		const uint32_t R = (uint32_t)rows.size();
		blk[7] = 4u * R;
		for (uint32_t h = 0; h < 2; ++h)
			for (uint32_t j = 0; j < R; ++j)
				blk.insert(blk.end(), rows[j]->begin() + 4 * h, rows[j]->begin() + 4 * h + 4);
	} else if (mode == 4u) {
		// single-candidate records, 16-B aligned, RW = 1 + ncls rounded up
		// to 4 words: w0 = constrained-class mask (bit 31: never holds),
		// w[1 + c] = what class c must be: the masked value (one-word
		// classes) or the key id (longer keys).  Compact form (more than 3
		// classes, but no alive rule constrains more than 3): RW = 4, the
		// values of the constrained classes in class order (w[1 + j] for the
		// j-th set bit of the mask) -- a quarter to a half of the bytes, so
		// larger rule sets keep their hot region in LDS
		bool compact = ncls > 3u;
		for (uint32_t r = 0; r < nrules && compact; ++r)
			if (alive[r] && __builtin_popcount(tmask[r]) > 3)
				compact = false;
		const uint32_t RW = compact ? 4u : (1u + ncls + 3u) & ~3u;
		align4();
		blk[4] = base + (uint32_t)blk.size();
		blk[5] = RW;
		uint32_t lk = prim_mask;
		for (uint32_t c = 0; c < ncls; ++c)
			if (cls_list[c].nkey > 1u)
				lk |= 1u << c;   // key ids for the record compare
		blk[6] = lk;
		blk[7] = prim_mask;
		for (uint32_t r = 0; r < nrules; ++r) {
			std::vector<uint32_t> rec(RW, 0);
			if (alive[r]) {
				rec[0] = tmask[r];
				uint32_t j = 0;
				for (uint32_t c = 0; c < ncls; ++c)
					if ((tmask[r] >> c) & 1u)
						rec[1 + (compact ? j++ : c)] = cls_list[c].nkey == 1u
							? want[r][c][0] : kid[c][want[r][c]];
			} else {
				rec[0] = 0x80000000u;
			}
			blk.insert(blk.end(), rec.begin(), rec.end());
		}
	} else if (mode == 1u) {
		const uint32_t RW = 1u + (ncls + 1u) / 2u;
		blk[4] = base + (uint32_t)blk.size();
		blk[5] = RW;
		for (uint32_t c = 0; c < ncls; ++c)
			lists[c].resize(kid[c].size() + 1);
		for (uint32_t r = 0; r < nrules; ++r) {
			std::vector<uint32_t> rec(RW, 0);
			if (alive[r]) {
				rec[0] = tmask[r];
				uint32_t prim = BV_NONE, best = 0xFFFFFFFFu;
				for (uint32_t c = 0; c < ncls; ++c) {
					if (!((tmask[r] >> c) & 1u))
						continue;
					rec[1 + c / 2] |= kid[c][want[r][c]] << (16 * (c & 1u));
					const uint32_t f = freq[c][want[r][c]];
					if (f < best) {
						best = f;
						prim = c;
					}
				}
				if (prim != BV_NONE)
					lists[prim][kid[prim][want[r][prim]]].push_back(r);
			} else {
				rec[0] = 0x80000000u;   // never holds
			}
			blk.insert(blk.end(), rec.begin(), rec.end());
		}
	}
	auto first_live = [&](uint32_t c, const Key4 *v) -> uint32_t {
		for (uint32_t r = 0; r < nrules; ++r)
			if (alive[r] && holds_class(r, c, v))
				return r;
		return BV_NONE;
	};
	auto row_of = [&](uint32_t c, const Key4 *v) -> uint32_t {
		uint32_t w = 0;
		for (uint32_t r = 0; r < nrules; ++r)
			if (holds_class(r, c, v))
				w |= 1u << r;
		return w;
	};
	for (uint32_t c = 0; c < ncls; ++c) {
		const ClassKey &ck = cls_list[c];
		std::vector<Key4> keys;
		for (auto &kv : kid[c])
			keys.push_back(kv.first);
		uint32_t nb = 1, m1 = 1, m2 = 3;   // bucket count, multipliers
		std::vector<uint32_t> slot_of;
		// one-word keys: 2-slot buckets of 16 B; longer keys: 1 slot per bucket
		const uint32_t bsz = ck.nkey == 1 ? 2u : 1u;
		if (!cuckoo_place(keys, ck.nkey, bsz, nb, m1, m2, slot_of))
			return false;
		const uint32_t cbase = 8 + BV_CLS_WORDS * c;
		const uint32_t ib = mode == 0u ? 2u : 8u + 8u * c;   // split class info
		std::array<uint32_t, 16> rec;
		rec.fill(0u);
		auto setc = [&](uint32_t w, uint32_t v) {
			if (split)
				rec[w] = v;
			else
				blk[cbase + w] = v;
		};
		// slot: key words, value; one-word keys 2 words (two slots per 16-B
		// bucket), 2-3-word keys one 16-B slot, 4-word keys 32 B
		const uint32_t SW = bsz == 2u ? 2u : (ck.nkey <= 3u ? 4u : 8u);
		setc(0, ck.kind);
		setc(1, ck.nkey);
		const uint32_t fl0 = mode == 0u ? first_live(c, nullptr) : 0u;
		const uint32_t miss = mode == 0u ? (fl0 == BV_NONE ? 0u : res_word(fl0) | BV_RES_VALID)
			: (mode == 2u ? row_of(c, nullptr) : (mode == 3u ? base + rows_at + 4u * miss_id[c] : 0u));
		if (split)
			blk[ib + 1] = miss;
		else
			blk[cbase + 2] = miss;
		setc(3, ck.offset);
		setc(4, ck.size);
		for (int i = 0; i < 4; ++i)
			setc(5 + i, ck.mask[i]);
		if (split) {
			blk[ib + 2] = nb;
			blk[ib + 4] = m1;
			blk[ib + 5] = m2;
		} else {
			blk[cbase + 9] = nb;
			blk[cbase + 11] = m1;
			blk[cbase + 12] = m2;
		}
		{
			const bool special = ck.kind == MI_K_LEN || ck.kind == MI_K_PCP0 ||
					     ck.kind == MI_K_DSCP;
			const FDesc d = fdesc(ck.kind, ck.offset);
			if (d.add > 0xffffu || d.alt > 0xffffu)
				return false;   // custom offset past 64 KiB: linear scan
			// "always present" (custom frame) is F_L2, which every parsed
			// frame has
			const uint32_t gate = d.gate == ~0u ? F_L2 : d.gate;
			const uint32_t ac = d.altf == F_QINQ ? 1u
				: (d.altf == F_IPV4 ? 2u : (d.altf == F_AH ? 3u : 0u));
			const uint32_t fl = (special ? BVF_SPECIAL : 0u) |
				((ck.kind == MI_K_CUSTOM_FRAME || ck.kind == MI_K_CUSTOM_L3) ? BVF_CUSTOM : 0u) |
				(ck.kind == MI_K_CUSTOM_L3 ? BVF_L3 : 0u) | (ck.kind == K_L4PORT ? BVF_TAG : 0u);
			setc(BVC_AO, d.add | (d.alt << 16));
			setc(BVC_DESC, (gate & 0xffffffu) | (d.base << 24) | (ac << 26) | (fl << 28));
		}
		if (split)
			shared.emplace_back(ib, rec);
		align4();   // 16-B buckets / slots
		const uint32_t tbl_off = (uint32_t)blk.size();
		if (split)
			blk[ib + 3] = base + tbl_off;
		else
			blk[cbase + 10] = base + tbl_off;
		// empty slots keep key words 0 and value 0: a miss (every stored
		// value is non-zero)
		blk.resize(blk.size() + (size_t)nb * bsz * SW, 0);
		uint32_t list_at = 0;
		if (mode == 1u) {
			blk[cbase + 13] = base + (uint32_t)blk.size();
			for (auto &l : lists[c]) {
				if (l.size() > 255u)
					return false;   // degenerate: the linear scan is cheaper
				blk.insert(blk.end(), l.begin(), l.end());
			}
			if (blk.size() - (blk[cbase + 13] - base) > 4095u)
				return false;
		}
		for (uint32_t i = 0; i < keys.size(); ++i) {
			const uint32_t sl = tbl_off + slot_of[i] * SW;
			for (uint32_t j = 0; j < ck.nkey; ++j)
				blk[sl + j] = keys[i][j];
			uint32_t val;
			if (mode == 0u) {
				const uint32_t f = first_live(c, &keys[i]);
				val = f == BV_NONE ? BV_EMPTY : res_word(f) | BV_RES_VALID;
			} else if (mode == 2u) {
				val = row_of(c, &keys[i]);   // non-zero: the key's own rules
			} else if (mode == 3u) {
				val = base + rows_at + 4u * key_row[c][i];   // word index, non-zero
			} else if (mode == 4u) {
				// key id << 16 | 1 + the rule filed under this key (0: none)
				uint32_t cand = 0;
				for (uint32_t r = 0; r < nrules && !cand; ++r)
					if (prim_of[r] == c && want[r][c] == keys[i])
						cand = r + 1u;
				val = (kid[c][keys[i]] << 16) | cand;
			} else {
				const uint32_t id = kid[c][keys[i]];
				uint32_t off = 0;
				for (uint32_t q = 0; q < id; ++q)
					off += (uint32_t)lists[c][q].size();
				val = id | ((uint32_t)lists[c][id].size() << 12) | (off << 20);
			}
			blk[sl + ck.nkey] = val;
		}
		(void)list_at;
	}
	return true;
}

// Assemble the mi_cls.h table into the private device encoding.
static int assemble(const void *tbl, uint32_t **out, size_t *out_words)
{
	const mi_tbl_hdr_t *h = (const mi_tbl_hdr_t *)tbl;
	const uint8_t *b = (const uint8_t *)tbl;
	const mi_cos_t *cs = (const mi_cos_t *)(b + h->cos_off);
	const mi_rule_t *rs = (const mi_rule_t *)(b + h->rule_off);
	const mi_term_t *ts = (const mi_term_t *)(b + h->term_off);
	// hot region: CoS table then the BV blocks (offsets relative to hot_off)
	std::vector<uint32_t> hot((size_t)COS_WORDS * h->num_cos, 0);
	for (uint32_t s = 0; s < h->num_cos; ++s) {
		uint32_t *c = &hot[COS_WORDS * s];
		c[C_NR] = cs[s].num_rules;
		c[C_META] = (uint32_t)cs[s].action | ((uint32_t)cs[s].num_queue << 8) |
			    ((uint32_t)cs[s].hash_proto << 16) | ((uint32_t)cs[s].index << 24);
		c[C_REC0] = cs[s].rule_begin;
	}
	if (!getenv("MI_CLS_NO_BV")) {
		// direct blocks' class records, one copy per distinct record
		std::map<std::array<uint32_t, 16>, std::vector<uint32_t>> shared_users;   // -> patch words
		for (uint32_t s = 0; s < h->num_cos; ++s) {
			if (!cs[s].valid || cs[s].num_rules == 0)
				continue;
			std::vector<uint32_t> blk;
			std::vector<std::pair<uint32_t, std::array<uint32_t, 16>>> shared;
			while (hot.size() & 3u)   // blocks start 16-B aligned (16-B row / bucket reads)
				hot.push_back(0);
			const uint32_t base = (uint32_t)hot.size();
			if (build_bv(cs, rs + cs[s].rule_begin, ts, cs[s].num_rules, base, blk, shared)) {
				hot[COS_WORDS * s + C_BV] = base;
				hot.insert(hot.end(), blk.begin(), blk.end());
				for (auto &sh : shared)
					shared_users[sh.second].push_back(base + sh.first);
			}
		}
		for (auto &kv : shared_users) {
			while (hot.size() & 3u)
				hot.push_back(0);
			const uint32_t at = (uint32_t)hot.size();
			hot.insert(hot.end(), kv.first.begin(), kv.first.end());
			for (uint32_t w : kv.second)
				hot[w] = at;
		}
	}
	// cold region: 16-word rule records (+ ext terms appended after them)
	const uint32_t hot_off = DH_WORDS;
	const size_t prog_off = hot_off + hot.size();
	std::vector<uint32_t> w(prog_off + (size_t)h->num_rules * REC_WORDS, 0);
	std::copy(hot.begin(), hot.end(), w.begin() + hot_off);
	w[DH_MAGIC] = DEV_MAGIC;
	w[DH_NCOS] = h->num_cos;
	w[DH_DEFAULT] = (uint32_t)h->default_cos;
	w[DH_ERROR] = (uint32_t)h->error_cos;
	w[DH_DEFAULT_VALID] = h->default_valid;
	w[DH_USED] = h->used_kinds;
	w[DH_MAX_HOPS] = h->max_hops;
	w[DH_HOT_OFF] = hot_off;
	w[DH_HOT_WORDS] = (uint32_t)hot.size();
	w[DH_PROG_OFF] = (uint32_t)prog_off;
	{
		// furthest bytes the terms read, per base (window predictor only:
		// correctness never depends on these)
		uint32_t end[3] = { 0, 0, 0 };
		for (uint32_t i = 0; i < h->num_terms; ++i) {
			const mi_term_t &t = ts[i];
			uint32_t base = FB_FRAME, e = 0;
			switch (t.kind) {
			case MI_K_LEN: case MI_K_NEVER: case MI_K_ALWAYS:
				break;
			case MI_K_PCP0: e = 16; break;
			case MI_K_DSCP: base = FB_L3; e = 4; break;
			case MI_K_CUSTOM_FRAME: e = t.offset + t.size + 4u; break;
			case MI_K_CUSTOM_L3: base = FB_L3; e = t.offset + t.size + 4u; break;
			default: {
				const FDesc d = fdesc(t.kind, 0);
				const uint32_t nw = (t.kind == MI_K_SIP6 || t.kind == MI_K_DIP6) ? 4u
					: (t.kind == MI_K_DMAC ? 2u : 1u);
				base = d.base;
				e = std::max(d.add, d.alt) + 4u * nw;
			}
			}
			end[base] = std::max(end[base], std::min(e, 0xFFFFu));
		}
		for (uint32_t s = 0; s < h->num_cos; ++s)
			if (cs[s].num_queue > 1) {   // Toeplitz tuple (rss_hash)
				end[FB_L3] = std::max(end[FB_L3], 40u);
				end[FB_L4] = std::max(end[FB_L4], 4u);
			}
		w[DH_FREND] = end[FB_FRAME];
		w[DH_L3END] = end[FB_L3];
		w[DH_L4END] = end[FB_L4];
	}
	std::vector<uint32_t> ext;
	const size_t ext_base = (size_t)h->num_rules * REC_WORDS;
	for (uint32_t r = 0; r < h->num_rules; ++r) {
		uint32_t *rec = &w[prog_off + (size_t)r * REC_WORDS];
		uint32_t used = 2, n_in = 0, n_ext = 0;
		size_t ext_begin = ext_base + ext.size();
		for (uint32_t t = 0; t < rs[r].num_terms; ++t) {
			uint32_t tw[12];
			uint32_t n = encode_term(ts[rs[r].term_begin + t], tw);
			if (n_ext == 0 && used + n <= REC_WORDS) {
				memcpy(rec + used, tw, n * sizeof(uint32_t));
				used += n;
				n_in++;
			} else {
				ext.insert(ext.end(), tw, tw + n);
				n_ext++;
			}
		}
		if (ext_begin >= (1u << 24))
			return -E2BIG;
		rec[0] = n_in | (n_ext << 8) | ((uint32_t)rs[r].mark << 16);
		rec[1] = rs[r].dst_cos | ((uint32_t)(n_ext ? ext_begin : 0) << 8);
	}
	w.insert(w.end(), ext.begin(), ext.end());
	w.resize(w.size() + 16, 0);
	w[DH_TOTAL] = (uint32_t)w.size();
	uint32_t *o = (uint32_t *)malloc(w.size() * sizeof(uint32_t));
	if (!o)
		return -ENOMEM;
	memcpy(o, w.data(), w.size() * sizeof(uint32_t));
	*out = o;
	*out_words = w.size();
	return 0;
}

// Host-only introspection of the device encoding a table assembles into (no
// device needed): info[0] total words, [1] hot-region words, [2] CoS with a
// classification block, [3..6] blocks per mode (direct, candidate, bitmap,
// wide), [7] 1 if the program is a tree (DIV kernel), [8] single-candidate
// blocks.  Tests and tools use it
// to check the engine choice on the CPU.
extern "C" int mi_cls_program_info(const void *tbl, size_t bytes, uint32_t *info, uint32_t n)
{
	if (!info || n < 9)
		return -EINVAL;
	int rc = validate_tbl(tbl, bytes);
	if (rc)
		return rc;
	uint32_t *w = nullptr;
	size_t words = 0;
	rc = assemble(tbl, &w, &words);
	if (rc)
		return rc;
	memset(info, 0, n * sizeof(uint32_t));
	info[0] = (uint32_t)words;
	info[1] = w[DH_HOT_WORDS];
	const mi_tbl_hdr_t *th = (const mi_tbl_hdr_t *)tbl;
	const uint32_t *hot = w + w[DH_HOT_OFF];
	for (uint32_t s = 0; s < th->num_cos; ++s) {
		const uint32_t bv = hot[COS_WORDS * s + C_BV];
		if (bv) {
			info[2]++;
			const uint32_t md = hot[bv];
			info[md == 4u ? 8u : 3u + (md & 3u)]++;
		}
	}
	const mi_cos_t *tc = (const mi_cos_t *)((const uint8_t *)tbl + th->cos_off);
	const mi_rule_t *tr = (const mi_rule_t *)((const uint8_t *)tbl + th->rule_off);
	for (uint32_t r = 0; r < th->num_rules && !info[7]; ++r)
		info[7] = tc[tr[r].dst_cos].num_rules != 0;
	free(w);
	return 0;
}

extern "C" int mi_cls_rules_load(mi_cls_ctx_t *c, const void *tbl, size_t bytes, void *stream)
{
	if (!c)
		return -EINVAL;
	int rc = validate_tbl(tbl, bytes);
	if (rc)
		return rc;
	uint32_t *w = nullptr;
	size_t words = 0;
	rc = assemble(tbl, &w, &words);
	if (rc)
		return rc;
	// host batches still in flight classify with the rules they were
	// submitted under
	if (c->stream && hipStreamSynchronize(c->stream) != hipSuccess) {
		free(w);
		return -EIO;
	}
	const uint32_t hot_words = w[DH_HOT_WORDS];
	int tree = 0;
	{
		// a rule whose destination has rules, or an error CoS with rules
		// next to a default CoS with rules: lanes of a wave may then sit on
		// different CoS with rules in one round
		const mi_tbl_hdr_t *th = (const mi_tbl_hdr_t *)tbl;
		const mi_cos_t *tc = (const mi_cos_t *)((const uint8_t *)tbl + th->cos_off);
		const mi_rule_t *tr = (const mi_rule_t *)((const uint8_t *)tbl + th->rule_off);
		for (uint32_t r = 0; r < th->num_rules && !tree; ++r)
			tree = tc[tr[r].dst_cos].num_rules != 0;
		if (th->error_cos >= 0 && th->default_cos >= 0 && tc[th->error_cos].num_rules &&
		    tc[th->default_cos].num_rules)
			tree = 1;
		const char *e = getenv("MI_CLS_DIV");
		if (e)
			tree = atoi(e) != 0;
		e = getenv("MI_CLS_WPB");
		c->wpb = e ? atoi(e) : 0;
	}
	int flat_mode = -1;
	{
		// flat program: the default CoS has a classification block and all
		// its rules lead to CoS without rules (one round decides every
		// packet); MI_CLS_NO_FLAT disables the flat kernels (A/B, tests)
		const mi_tbl_hdr_t *th = (const mi_tbl_hdr_t *)tbl;
		const mi_cos_t *tc = (const mi_cos_t *)((const uint8_t *)tbl + th->cos_off);
		const mi_rule_t *tr = (const mi_rule_t *)((const uint8_t *)tbl + th->rule_off);
		const int32_t d = th->default_cos;
		if (d >= 0 && th->default_valid && tc[d].num_rules && !getenv("MI_CLS_NO_FLAT")) {
			const uint32_t *hot = w + w[DH_HOT_OFF];
			const uint32_t bv = hot[COS_WORDS * (uint32_t)d + C_BV];
			bool leaves = true;
			for (uint32_t r = 0; r < tc[d].num_rules && leaves; ++r)
				leaves = tc[tr[tc[d].rule_begin + r].dst_cos].num_rules == 0;
			if (bv && leaves && hot[bv] != 1u)
				flat_mode = (int)hot[bv];
		}
	}
	if (getenv("MI_CLS_VERBOSE"))
		fprintf(stderr, "mi_cls: program %zu words, hot region %u words\n", words, hot_words);
	size_t nbytes = words * sizeof(uint32_t);
	if (hipSetDevice(c->device) != hipSuccess)
		return free(w), -EIO;
	if (nbytes > c->dev_cap) {
		// the old program may still be read by in-flight launches
		if (c->d_dev) {
			if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
				return free(w), -EIO;
			(void)hipFree(c->d_dev);
			c->d_dev = nullptr;
		}
		size_t cap = nbytes < 4096 ? 4096 : nbytes;
		if (hipMalloc((void **)&c->d_dev, cap) != hipSuccess)
			return free(w), -ENOMEM;
		c->dev_cap = cap;
	}
	// stream-ordered after earlier launches; synchronous w.r.t. the host
	// buffer, which is freed on return
	hipError_t e = hipMemcpyAsync(c->d_dev, w, nbytes, hipMemcpyHostToDevice, (hipStream_t)stream);
	if (e == hipSuccess)
		e = hipStreamSynchronize((hipStream_t)stream);
	free(w);
	if (e != hipSuccess)
		return -EIO;
	c->hot_words = hot_words;
	c->tree = tree;
	c->flat_mode = flat_mode;
	c->loaded = 1;
	return 0;
}

extern "C" int mi_cls_classify(mi_cls_ctx_t *c, const uint8_t *pkts, const uint32_t *off,
			       const uint16_t *len, uint32_t n, mi_cls_result_t *out, void *stream)
{
	if (!c || !c->loaded)
		return -EINVAL;
	if (n == 0)
		return 0;
	if (!pkts || !off || !len || !out)
		return -EINVAL;
	if (((uintptr_t)out & 15u) != 0)
		return -EINVAL;
	HIP_OK(hipSetDevice(c->device));
	KArgs a;
	a.pkts = pkts;
	a.off = off;
	a.len = len;
	a.n = n;
	a.dev = c->d_dev;
	a.out = out;
	a.stats = c->stats_on ? c->d_stats : nullptr;
	a.diag = nullptr;
	a.opt = c->opt;
	a.hint = c->d_hint;
	a.seq = ++c->seq;
	if (a.seq == 0u)   // wrapped: the hint word may equal seq - 1 by accident
		a.seq = c->seq = 2u;
#ifdef DIAG_STAMPS
	static unsigned long long *d_diag = nullptr;
	if (!d_diag)
		(void)hipMalloc((void **)&d_diag, 16 * sizeof(unsigned long long));
	(void)hipMemset(d_diag, 0, 16 * sizeof(unsigned long long));
	a.diag = d_diag;
#endif
	memcpy(a.stats_mask, c->stats_mask, sizeof(a.stats_mask));
	// One wave per 64-packet tile in flight; the grid covers the resident
	// capacity (blocks per CU: 4 = the VGPR-bound occupancy of 4 waves/SIMD,
	// fewer when the LDS copy of the hot region does not leave room) and each
	// wave loops over its tiles with the load pipeline.
	// MI_CLS_BLOCKS_PER_CU overrides the block count, MI_CLS_LDS_HOT_MAX
	// (bytes) the largest hot region copied into LDS.
	static int per_cu_env = -2, hot_max = -1;
	if (per_cu_env == -2) {
		const char *e = getenv("MI_CLS_BLOCKS_PER_CU");
		per_cu_env = e ? atoi(e) : -1;
		e = getenv("MI_CLS_LDS_HOT_MAX");
		hot_max = e ? atoi(e) : 20 * 1024;
	}
	// Block shape: 4-wave blocks, four per CU, each with its own LDS copy of
	// the hot region when it is small (<= MI_CLS_LDS_HOT_MAX); otherwise one
	// block per CU of 16, 12 or 8 waves sharing one copy -- the most waves
	// whose windows leave room for it; otherwise 4-wave blocks reading the
	// hot region from HBM.  MI_CLS_WPB=4|8|12|16 forces a shape (A/B runs).
	const int wpb_env = c->wpb;
	const size_t LDS_CU = 160u * 1024u;
	const size_t hot_bytes = (((size_t)c->hot_words + 3u) & ~(size_t)3u) * sizeof(uint32_t);
	// static LDS of a block: windows, stats histogram, L4 table (+ the
	// CRC-32C tables of the pktin-option kernels)
	const size_t st_ck = c->opt != 0 ? 1024 + CRC_ZN + 64 : 0;
	auto st_of = [st_ck](int w) {
		return sizeof(uint32_t) * ((size_t)w * RS * WROWS + MAX_STATS_COS + 256 + st_ck);
	};
	const bool small = (long)hot_bytes <= (long)hot_max;
	const bool full4 = small && 4 * (st_of(4) + hot_bytes) <= LDS_CU;
	int nw = 4;
	bool lt = full4;
	if (!full4) {
		for (int w : { 16, 12, 8 })
			if (st_of(w) + hot_bytes <= LDS_CU) {
				nw = w;
				lt = true;
				break;
			}
	}
	if (wpb_env == 4 || wpb_env == 8 || wpb_env == 12 || wpb_env == 16) {
		nw = wpb_env;
		lt = nw == 4 ? small && st_of(4) + hot_bytes <= LDS_CU : st_of(nw) + hot_bytes <= LDS_CU;
		if (nw != 4 && nw != 16 && !lt)
			nw = 16;   // 8 / 12-wave blocks exist for LDS-resident hot regions only
	}
	if (c->opt != 0 && nw != 4) {
		// the pktin-option kernels exist as 4-wave blocks and as 16-wave
		// blocks with the hot region in LDS
		nw = 16;
		lt = st_of(16) + hot_bytes <= LDS_CU;
		if (!lt)
			nw = 4;
	}
	const size_t lds_block = st_of(nw) + (lt ? hot_bytes : 0);
	const bool div = c->tree;
	int per_cu = (int)(LDS_CU / lds_block);
	const int occ = MIN_WAVES_PER_EU;   // waves/SIMD the register budget allows
	if (per_cu > occ * 4 / nw)
		per_cu = occ * 4 / nw;
	if (per_cu_env > 0)
		per_cu = per_cu_env;
	if (per_cu < 1)
		per_cu = 1;
	const uint32_t bthreads = (uint32_t)nw * WAVE;
	uint32_t tiles = (n + bthreads - 1) / bthreads;
	uint32_t max_grid = (uint32_t)c->num_cu * (uint32_t)per_cu;
	uint32_t grid = tiles < max_grid ? tiles : max_grid;
	const size_t dyn = lt ? hot_bytes : 0;
	hipStream_t st = (hipStream_t)stream;
	int lrc;
	if (c->opt != 0)
		lrc = mi_cls_launch_ck(nw, lt, div, grid, dyn, st, a);
	else if (c->flat_mode >= 0 && lt && (nw == 4 || nw == 12 || nw == 16))
		lrc = mi_cls_launch_flat(nw, c->flat_mode, grid, dyn, st, a);
	else if (nw == 16)
		lrc = mi_cls_launch_k16(lt, div, grid, dyn, st, a);
	else if (nw == 12)
		lrc = mi_cls_launch_k12(lt, div, grid, dyn, st, a);
	else if (nw == 8)
		lrc = mi_cls_launch_k8(lt, div, grid, dyn, st, a);
	else
		lrc = mi_cls_launch_k4(lt, div, grid, dyn, st, a);
	if (lrc)
		return lrc;
	if (hipGetLastError() != hipSuccess)
		return -EIO;
#ifdef DIAG_STAMPS
	{
		unsigned long long h[16];
		(void)hipStreamSynchronize((hipStream_t)stream);
		(void)hipMemcpy(h, d_diag, sizeof(h), hipMemcpyDeviceToHost);
		fprintf(stderr, "DIAG waves=%llu cycles/wave:", h[8]);
		for (int i = 0; i < 8; ++i)
			fprintf(stderr, " p%d=%.0f", i, (double)h[i] / (double)(h[8] ? h[8] : 1));
		fprintf(stderr, "\n");
	}
#endif
	return 0;
}

// Stage frames [lo, hi) of a host batch (descriptors rebased by lo) through
// the context's device buffers on its own stream and launch the kernel; the
// records go to `out` (any host memory) or, when out is NULL, to the
// context's pinned record buffer h_out (multi-GPU: no host wait per device).
// Nothing is waited for here.
// Device address of page-locked host memory (hipHostMalloc /
// hipHostRegister), NULL for pageable memory.
static const void *dev_view(const void *p)
{
	hipPointerAttribute_t a;
	if (hipPointerGetAttributes(&a, p) != hipSuccess) {
		(void)hipGetLastError();
		return nullptr;
	}
	if (a.type != hipMemoryTypeHost || !a.devicePointer || !a.hostPointer)
		return nullptr;
	return (const uint8_t *)a.devicePointer + ((const uint8_t *)p - (const uint8_t *)a.hostPointer);
}

// `lim` is the size of the caller's buffer at `pkts`: the zero-copy path is
// taken only when every frame's last 16-B piece (the kernel reads frames in
// 16-B pieces from their start) lies inside it; otherwise the frames are
// staged into the padded device buffer.
static int host_launch(mi_cls_ctx_t *c, const uint8_t *pkts, size_t lo, size_t hi, size_t lim,
		       const uint32_t *off, const uint16_t *len, uint32_t n, mi_cls_result_t *out)
{
	HIP_OK(hipSetDevice(c->device));
	if (!c->stream)
		HIP_OK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
	// Zero copy: frames and descriptors in page-locked memory are read by the
	// kernel in place over the host link -- only the header windows it
	// touches cross it, not whole frames -- and the records are written
	// straight into page-locked `out`.
	const void *zp = dev_view(pkts), *zo = zp ? dev_view(off) : nullptr;
	const void *zl = zo ? dev_view(len) : nullptr;
	for (uint32_t i = 0; zl && i < n; ++i)
		if ((size_t)off[i] + (((size_t)len[i] + 15u) & ~(size_t)15u) > lim)
			zl = nullptr;
	if (zl) {
		mi_cls_result_t *o = out ? out : n <= c->n_cap ? c->h_out : nullptr;
		const void *zr = o ? dev_view(o) : nullptr;
		if (zr)   // descriptors keep their offsets relative to `pkts`
			return mi_cls_classify(c, (const uint8_t *)zp, (const uint32_t *)zo,
					       (const uint16_t *)zl, n, (mi_cls_result_t *)zr, c->stream);
	}
	const size_t bytes = hi - lo;
	const size_t need = bytes + 64;
	if ((need > c->pk_cap || n > c->n_cap) && c->submitted)
		HIP_OK(hipStreamSynchronize(c->stream));   // buffers of submitted batches
	if (need > c->pk_cap) {
		(void)hipFree(c->d_pk);
		c->d_pk = nullptr;
		size_t cap = need < (1u << 20) ? (1u << 20) : need + need / 2;
		if (hipMalloc((void **)&c->d_pk, cap) != hipSuccess)
			return c->pk_cap = 0, -ENOMEM;
		HIP_OK(hipMemset(c->d_pk, 0, cap));
		c->pk_cap = cap;
	}
	if (n > c->n_cap) {
		(void)hipFree(c->d_off);
		(void)hipFree(c->d_len);
		(void)hipFree(c->d_out);
		(void)hipHostFree(c->h_off);
		(void)hipHostFree(c->h_out);
		c->d_off = nullptr;
		c->d_len = nullptr;
		c->d_out = nullptr;
		c->h_off = nullptr;
		c->h_out = nullptr;
		uint32_t cap = n < 4096u ? 4096u : n + n / 2;
		if (hipMalloc((void **)&c->d_off, cap * sizeof(uint32_t)) != hipSuccess ||
		    hipMalloc((void **)&c->d_len, cap * sizeof(uint16_t)) != hipSuccess ||
		    hipMalloc((void **)&c->d_out, cap * sizeof(mi_cls_result_t)) != hipSuccess ||
		    hipHostMalloc((void **)&c->h_off, cap * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
		    hipHostMalloc((void **)&c->h_out, cap * sizeof(mi_cls_result_t), hipHostMallocDefault) != hipSuccess)
			return c->n_cap = 0, -ENOMEM;
		c->n_cap = cap;
	}
	hipStream_t s = c->stream;
	const uint32_t *doff = off;
	if (lo) {
		for (uint32_t i = 0; i < n; ++i)
			c->h_off[i] = off[i] - (uint32_t)lo;
		doff = c->h_off;
	}
	HIP_OK(hipMemcpyAsync(c->d_pk, pkts + lo, bytes, hipMemcpyHostToDevice, s));
	HIP_OK(hipMemcpyAsync(c->d_off, doff, n * sizeof(uint32_t), hipMemcpyHostToDevice, s));
	HIP_OK(hipMemcpyAsync(c->d_len, len, n * sizeof(uint16_t), hipMemcpyHostToDevice, s));
	int rc = mi_cls_classify(c, c->d_pk, c->d_off, c->d_len, n, c->d_out, s);
	if (rc)
		return rc;
	HIP_OK(hipMemcpyAsync(out ? out : c->h_out, c->d_out, n * sizeof(mi_cls_result_t),
			      hipMemcpyDeviceToHost, s));
	return 0;
}

// Host-memory batch: stage through device buffers owned by the context on its
// own stream (grown geometrically, kept across calls), classify, copy back.
extern "C" int mi_cls_classify_host(mi_cls_ctx_t *c, const uint8_t *pkts, size_t bytes,
				    const uint32_t *off, const uint16_t *len, uint32_t n,
				    mi_cls_result_t *out)
{
	if (!c || !c->loaded)
		return -EINVAL;
	if (n == 0)
		return 0;
	if (!pkts || !off || !len || !out)
		return -EINVAL;
	// every frame must lie inside the staged bytes (the kernel reads up to
	// the next 16-byte boundary after a frame; the staging buffer is padded)
	for (uint32_t i = 0; i < n; ++i)
		if ((size_t)off[i] + len[i] > bytes)
			return -EINVAL;
	int rc = host_launch(c, pkts, 0, bytes, bytes, off, len, n, out);
	if (rc)
		return rc;
	HIP_OK(hipStreamSynchronize(c->stream));
	return 0;
}

// Submit a host batch without waiting (pipelined receive): the caller keeps
// pkts / off / len / out untouched until mi_cls_classify_host_wait(ticket).
extern "C" int mi_cls_classify_host_submit(mi_cls_ctx_t *c, const uint8_t *pkts, size_t bytes,
					   const uint32_t *off, const uint16_t *len, uint32_t n,
					   mi_cls_result_t *out, uint64_t *ticket)
{
	if (!c || !c->loaded || !ticket)
		return -EINVAL;
	*ticket = 0;
	if (n == 0)
		return 0;
	if (!pkts || !off || !len || !out)
		return -EINVAL;
	for (uint32_t i = 0; i < n; ++i)
		if ((size_t)off[i] + len[i] > bytes)
			return -EINVAL;
	const uint64_t t = c->submitted + 1;
	hipEvent_t *ev = &c->ev[t % 8];
	HIP_OK(hipSetDevice(c->device));
	if (!*ev)
		HIP_OK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
	else
		HIP_OK(hipEventSynchronize(*ev));   // ticket t - 8: done before its slot is reused
	int rc = host_launch(c, pkts, 0, bytes, bytes, off, len, n, out);
	if (rc)
		return rc;
	HIP_OK(hipEventRecord(*ev, c->stream));
	c->submitted = t;
	*ticket = t;
	return 0;
}

extern "C" int mi_cls_classify_host_wait(mi_cls_ctx_t *c, uint64_t ticket)
{
	if (!c || ticket > c->submitted)
		return -EINVAL;
	if (ticket == 0 || ticket + 8 <= c->submitted)
		return 0;   // nothing submitted, or its slot was reused (waited for then)
	HIP_OK(hipSetDevice(c->device));
	HIP_OK(hipEventSynchronize(c->ev[ticket % 8]));
	return 0;
}

// ---------------------------------------------------------------- multi-GPU
// the batch shards with no exchange step.  Contiguous
// slices balanced by the bytes the kernel reads per packet (min(len,128) +
// 6 B descriptor + 16 B record), one per device; concatenating the slices'
// records in device order is the single-device result, so per-queue arrival
// order is what the reference's _odp_cls_enq runs see
// (odp_classification_internal.h:208-236).
extern "C" int mi_cls_shard(const uint16_t *len, uint32_t n, uint32_t nshards, uint32_t *begin)
{
	if (!begin || nshards == 0 || (n && !len))
		return -EINVAL;
	uint64_t total = 0;
	for (uint32_t i = 0; i < n; ++i)
		total += (uint64_t)(len[i] < 128u ? len[i] : 128u) + 22u;
	begin[0] = 0;
	uint64_t cum = 0;
	uint32_t i = 0;
	for (uint32_t r = 1; r < nshards; ++r) {
		// first packet index whose running total reaches r/nshards of the
		// whole; the cut follows it
		while (i < n && (cum + (uint64_t)(len[i] < 128u ? len[i] : 128u) + 22u) * nshards <
				       total * r) {
			cum += (uint64_t)(len[i] < 128u ? len[i] : 128u) + 22u;
			++i;
		}
		begin[r] = i < n ? i + 1u : n;
		if (begin[r] < begin[r - 1])
			begin[r] = begin[r - 1];
	}
	begin[nshards] = n;
	for (uint32_t r = 1; r < nshards; ++r)
		if (begin[r] > n)
			begin[r] = n;
	return 0;
}

#define MI_GROUP_MAX 64
struct mi_cls_group {
	uint32_t n;
	mi_cls_ctx_t *ctx[MI_GROUP_MAX];
	uint32_t *begin;          // nshards + 1
};

extern "C" int mi_cls_group_create(const int *devices, uint32_t n, mi_cls_group_t **out)
{
	if (!devices || !out || n == 0 || n > MI_GROUP_MAX)
		return -EINVAL;
	mi_cls_group_t *g = (mi_cls_group_t *)calloc(1, sizeof(*g));
	if (!g)
		return -ENOMEM;
	g->begin = (uint32_t *)calloc(n + 1, sizeof(uint32_t));
	if (!g->begin) {
		free(g);
		return -ENOMEM;
	}
	for (uint32_t i = 0; i < n; ++i) {
		int rc = mi_cls_ctx_create(devices[i], &g->ctx[i]);
		if (rc) {
			g->n = i;
			mi_cls_group_destroy(g);
			return rc;
		}
	}
	g->n = n;
	*out = g;
	return 0;
}

extern "C" int mi_cls_group_destroy(mi_cls_group_t *g)
{
	if (!g)
		return -EINVAL;
	for (uint32_t i = 0; i < g->n; ++i)
		mi_cls_ctx_destroy(g->ctx[i]);
	free(g->begin);
	free(g);
	return 0;
}

extern "C" uint32_t mi_cls_group_size(const mi_cls_group_t *g)
{
	return g ? g->n : 0u;
}

extern "C" mi_cls_ctx_t *mi_cls_group_ctx(mi_cls_group_t *g, uint32_t i)
{
	return g && i < g->n ? g->ctx[i] : nullptr;
}

extern "C" int mi_cls_group_rules_load(mi_cls_group_t *g, const void *tbl, size_t bytes)
{
	if (!g)
		return -EINVAL;
	for (uint32_t i = 0; i < g->n; ++i) {
		int rc = mi_cls_rules_load(g->ctx[i], tbl, bytes, nullptr);
		if (rc)
			return rc;
	}
	return 0;
}

extern "C" int mi_cls_group_pktin_opt_set(mi_cls_group_t *g, uint64_t opt)
{
	if (!g)
		return -EINVAL;
	for (uint32_t i = 0; i < g->n; ++i)
		mi_cls_pktin_opt_set(g->ctx[i], opt);
	return 0;
}

extern "C" int mi_cls_group_classify_host(mi_cls_group_t *g, const uint8_t *pkts, size_t bytes,
					  const uint32_t *off, const uint16_t *len, uint32_t n,
					  mi_cls_result_t *out)
{
	if (!g)
		return -EINVAL;
	if (n == 0)
		return 0;
	if (!pkts || !off || !len || !out)
		return -EINVAL;
	for (uint32_t k = 0; k < g->n; ++k)
		if (!g->ctx[k]->loaded)
			return -EINVAL;
	for (uint32_t i = 0; i < n; ++i)
		if ((size_t)off[i] + len[i] > bytes)
			return -EINVAL;
	int rc = mi_cls_shard(len, n, g->n, g->begin);
	if (rc)
		return rc;
	// every device's slice in flight before any wait.  Page-locked batches
	// are read in place (host_launch only enqueues work), so one thread
	// launches every slice; a pageable batch is staged by a copy the HIP
	// runtime performs synchronously, so each device gets its own host
	// thread and the slices' copies run side by side.
	int err[MI_GROUP_MAX] = { 0 };
	auto run = [&](uint32_t k, bool wait) {
		const uint32_t b = g->begin[k], e = g->begin[k + 1];
		if (b == e)
			return;
		size_t lo = off[b], hi = 0;
		for (uint32_t i = b; i < e; ++i) {
			lo = off[i] < lo ? off[i] : lo;
			hi = (size_t)off[i] + len[i] > hi ? (size_t)off[i] + len[i] : hi;
		}
		lo &= ~(size_t)15;   // keep the slice's 16-B alignment
		err[k] = host_launch(g->ctx[k], pkts, lo, hi, bytes, off + b, len + b, e - b, nullptr);
		if (err[k] || !wait)
			return;
		if (hipSetDevice(g->ctx[k]->device) != hipSuccess ||
		    hipStreamSynchronize(g->ctx[k]->stream) != hipSuccess) {
			err[k] = -EIO;
			return;
		}
		memcpy(out + b, g->ctx[k]->h_out, (size_t)(e - b) * sizeof(mi_cls_result_t));
	};
	if (dev_view(pkts) || g->n == 1) {
		for (uint32_t k = 0; k < g->n; ++k)
			run(k, false);
		for (uint32_t k = 0; k < g->n; ++k) {
			const uint32_t b = g->begin[k], e = g->begin[k + 1];
			if (b == e || err[k])
				continue;
			if (hipSetDevice(g->ctx[k]->device) != hipSuccess ||
			    hipStreamSynchronize(g->ctx[k]->stream) != hipSuccess) {
				err[k] = -EIO;
				continue;
			}
			memcpy(out + b, g->ctx[k]->h_out, (size_t)(e - b) * sizeof(mi_cls_result_t));
		}
	} else {
		std::vector<std::thread> th;
		for (uint32_t k = 1; k < g->n; ++k)
			th.emplace_back(run, k, true);
		run(0, true);
		for (auto &t : th)
			t.join();
	}
	for (uint32_t k = 0; k < g->n; ++k)
		if (err[k])
			return err[k];
	return 0;
}

// pktin options for the following classify calls: odp_pktin_config_opt_t
// all_bits (checksum validation and drop-on-error bits; timestamps ignored).
extern "C" int mi_cls_pktin_opt_set(mi_cls_ctx_t *c, uint64_t opt)
{
	if (!c)
		return -EINVAL;
	c->opt = (uint32_t)(opt & 0x7FCull);   // bits 2..10
	return 0;
}

extern "C" void *mi_cls_host_alloc(size_t bytes)
{
	void *p = nullptr;
	if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable | hipHostMallocMapped) != hipSuccess)
		return nullptr;
	return p;
}

extern "C" void mi_cls_host_free(void *p)
{
	if (p)
		(void)hipHostFree(p);
}

extern "C" int mi_cls_stats_enable(mi_cls_ctx_t *c, const uint32_t mask[8])
{
	if (!c)
		return -EINVAL;
	int any = 0;
	for (int i = 0; i < 8; ++i) {
		c->stats_mask[i] = mask ? mask[i] : 0u;
		any |= c->stats_mask[i] != 0;
	}
	c->stats_on = any;
	return 0;
}

extern "C" int mi_cls_stats_read(mi_cls_ctx_t *c, uint64_t *host, uint32_t num)
{
	if (!c || !host || num > MAX_STATS_COS)
		return -EINVAL;
	HIP_OK(hipSetDevice(c->device));
	HIP_OK(hipDeviceSynchronize());
	HIP_OK(hipMemcpy(host, c->d_stats, num * sizeof(uint64_t), hipMemcpyDeviceToHost));
	return 0;
}

extern "C" int mi_cls_stats_reset(mi_cls_ctx_t *c)
{
	if (!c)
		return -EINVAL;
	HIP_OK(hipSetDevice(c->device));
	HIP_OK(hipDeviceSynchronize());
	HIP_OK(hipMemset(c->d_stats, 0, MAX_STATS_COS * sizeof(unsigned long long)));
	return 0;
}

extern "C" const char *mi_cls_strerror(int err)
{
	switch (-err) {
	case 0: return "success";
	case EINVAL: return "invalid argument or malformed rule table";
	case ENODEV: return "no such HIP device";
	case ENOMEM: return "out of device memory";
	case EIO: return "HIP runtime error";
	default: return "unknown error";
	}
}
