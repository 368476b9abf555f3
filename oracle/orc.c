/*
 * orc.c - CPU oracle for the rx classify path.  TEST INFRASTRUCTURE ONLY:
 * linked by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
 * never by the product.  See orc.h for what each function restates.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "orc.h"

#define ROT(x, k) (((x) << (k)) | ((x) >> (32 - (k))))

/* lookup3 mix/final, base/jenkins_hash.c:79-87 and :114-123 */
#define MIX(a, b, c) do { \
	a -= c; a ^= ROT(c, 4);  c += b; \
	b -= a; b ^= ROT(a, 6);  a += c; \
	c -= b; c ^= ROT(b, 8);  b += a; \
	a -= c; a ^= ROT(c, 16); c += b; \
	b -= a; b ^= ROT(a, 19); a += c; \
	c -= b; c ^= ROT(b, 4);  b += a; \
} while (0)
#define FINAL(a, b, c) do { \
	c ^= b; c -= ROT(b, 14); \
	a ^= c; a -= ROT(c, 11); \
	b ^= a; b -= ROT(a, 25); \
	c ^= b; c -= ROT(b, 16); \
	a ^= c; a -= ROT(c, 4);  \
	b ^= a; b -= ROT(a, 14); \
	c ^= b; c -= ROT(b, 24); \
} while (0)

/*
 * orc_jhash - lookup3 hashlittle with initval 0 (base/jenkins_hash.c:126-297).
 * Restated on the byte-at-a-time branch (:252-293), which yields the same
 * value as the aligned branches for every input.
 */
uint32_t orc_jhash(const void *key, size_t len)
{
	const uint8_t *k = key;
	uint32_t a, b, c;

	a = b = c = 0xdeadbeefu + (uint32_t)len;
	while (len > 12) {
		a += k[0] | (uint32_t)k[1] << 8 | (uint32_t)k[2] << 16 | (uint32_t)k[3] << 24;
		b += k[4] | (uint32_t)k[5] << 8 | (uint32_t)k[6] << 16 | (uint32_t)k[7] << 24;
		c += k[8] | (uint32_t)k[9] << 8 | (uint32_t)k[10] << 16 | (uint32_t)k[11] << 24;
		MIX(a, b, c);
		len -= 12;
		k += 12;
	}
	switch (len) {
	case 12: c += (uint32_t)k[11] << 24; /* fall through */
	case 11: c += (uint32_t)k[10] << 16; /* fall through */
	case 10: c += (uint32_t)k[9] << 8;   /* fall through */
	case 9:  c += k[8];                  /* fall through */
	case 8:  b += (uint32_t)k[7] << 24;  /* fall through */
	case 7:  b += (uint32_t)k[6] << 16;  /* fall through */
	case 6:  b += (uint32_t)k[5] << 8;   /* fall through */
	case 5:  b += k[4];                  /* fall through */
	case 4:  a += (uint32_t)k[3] << 24;  /* fall through */
	case 3:  a += (uint32_t)k[2] << 16;  /* fall through */
	case 2:  a += (uint32_t)k[1] << 8;   /* fall through */
	case 1:  a += k[0]; break;
	case 0:  return c; /* zero length: no mixing, :180 */
	}
	FINAL(a, b, c);
	return c;
}

static inline uint32_t be32_of(const uint8_t *p)
{
	return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

/*
 * orc_do_toeplitz - runtime/net/core.c:120-139.  Input words are
 * {saddr, daddr, dport | sport << 16} in host order; for every set bit i of
 * word j the 32-bit key window starting at that bit is xor-ed in.
 */
uint32_t orc_do_toeplitz(const uint8_t *key, uint32_t saddr, uint32_t daddr,
                         uint16_t sport, uint16_t dport)
{
	uint32_t in[3] = { saddr, daddr, (uint32_t)dport | (uint32_t)sport << 16 };
	uint32_t ret = 0;

	for (int j = 0; j < 3; j++) {
		uint32_t kj = be32_of(key + 4 * j), kj1 = be32_of(key + 4 * j + 4);
		for (uint32_t map = in[j]; map; map &= map - 1) {
			uint32_t i = (uint32_t)__builtin_ctz(map);
			ret ^= kj << (31 - i) | (uint32_t)((uint64_t)kj1 >> (i + 1));
		}
	}
	return ret;
}

/* Textbook Toeplitz over a byte string, MSB first (MS RSS verification). */
uint32_t orc_toeplitz_bytes(const uint8_t *key, size_t keylen,
                            const uint8_t *in, size_t len)
{
	uint32_t ret = 0;
	for (size_t p = 0; p < len * 8; p++) {
		if (!(in[p / 8] & (0x80 >> (p % 8))))
			continue;
		uint32_t w = 0;
		for (int q = 0; q < 32; q++) {
			size_t kb = p + q;
			int bit = kb / 8 < keylen ? (key[kb / 8] >> (7 - kb % 8)) & 1 : 0;
			w = w << 1 | (uint32_t)bit;
		}
		ret ^= w;
	}
	return ret;
}

/*
 * orc_crc32c_u64 - the crc32q instruction behind hash_crc32c_one/two
 * (inc/base/hash.h:23-40, inc/asm/ops.h:77-80): CRC32C, reflected polynomial
 * 0x82F63B78, over the 8 little-endian bytes of @val, no pre/post inversion.
 * Bit-serial restatement; pinned against the reference's own inline
 * functions compiled into oracle/_ref/libcrc_ref.so.
 */
uint32_t orc_crc32c_u64(uint32_t crc, uint64_t val)
{
	for (int bit = 0; bit < 64; bit++) {
		uint32_t in = (uint32_t)(val >> bit) & 1u;
		uint32_t fb = (crc ^ in) & 1u;
		crc >>= 1;
		if (fb)
			crc ^= 0x82F63B78u;
	}
	return crc;
}

/* sched_steer_flows, iokernel/sched.c:122-147 */
void orc_steer_flows(uint16_t thread_count, const uint16_t *active_idx,
                     uint16_t active_count, uint16_t *flow_tbl)
{
	int j = 0;

	if (active_count == 0)
		return;
	memset(flow_tbl, 0xFF, sizeof(*flow_tbl) * thread_count);
	for (int i = 0; i < active_count; i++)
		flow_tbl[active_idx[i]] = active_idx[i];
	for (int i = 0; i < thread_count; i++) {
		if (flow_tbl[i] != UINT16_MAX)
			continue;
		flow_tbl[i] = active_idx[j++ % active_count];
	}
}

/* ------------------------------------------------------------------------
 * IP -> runtime map.  Same contract as the rte_hash in dp_clients.c:349-363
 * (exact match on the 4-byte host-order IP, hashed with jhash initval 0);
 * laid out as 8-way buckets with a primary and an alternative bucket like
 * DPDK's cuckoo table, so the CPU baseline pays a comparable lookup.
 */
#define ORC_BKT 8
struct orc_bucket {
	uint32_t sig[ORC_BKT];
	uint32_t ip[ORC_BKT];
	int32_t  uid[ORC_BKT];
};

struct orc_tables {
	uint32_t max_runtimes;
	uint32_t hash_mode;
	uint32_t flags;
	uint8_t  default_olflags;
	uint8_t  rss_key[40];
	struct orc_runtime *rt;     /* [max_runtimes] = dp.clients_by_id */
	uint32_t *trans_seed;       /* [max_runtimes] runtime trans_seed */
	struct orc_bucket *bkt;
	uint32_t nbkt_mask;
};

static uint32_t alt_bucket(uint32_t h, uint32_t mask)
{
	return (h ^ ((h >> 16) | 1u) * 0x9E3779B1u) & mask;
}

struct orc_tables *orc_tables_new(uint32_t max_runtimes, uint32_t hash_mode,
                                  uint32_t flags, uint8_t default_olflags,
                                  const uint8_t *rss_key40)
{
	struct orc_tables *t;
	uint32_t nb = 2;

	if (max_runtimes == 0 || max_runtimes > GCL_MAX_PROC)
		return NULL;
	t = calloc(1, sizeof(*t));
	if (!t)
		return NULL;
	t->max_runtimes = max_runtimes;
	t->hash_mode = hash_mode;
	t->flags = flags;
	t->default_olflags = default_olflags;
	if (rss_key40)
		memcpy(t->rss_key, rss_key40, 40);
	t->rt = calloc(max_runtimes, sizeof(*t->rt));
	t->trans_seed = calloc(max_runtimes, sizeof(uint32_t));
	while (nb * ORC_BKT < 2 * max_runtimes)
		nb <<= 1;
	t->bkt = malloc(nb * sizeof(*t->bkt));
	if (!t->rt || !t->bkt) {
		orc_tables_free(t);
		return NULL;
	}
	for (uint32_t i = 0; i < nb; i++)
		for (int s = 0; s < ORC_BKT; s++)
			t->bkt[i].uid[s] = -1;
	t->nbkt_mask = nb - 1;
	return t;
}

void orc_tables_free(struct orc_tables *t)
{
	if (!t)
		return;
	free(t->rt);
	free(t->trans_seed);
	free(t->bkt);
	free(t);
}

static int iptab_lookup(const struct orc_tables *t, uint32_t ip)
{
	uint32_t h = orc_jhash(&ip, 4);
	uint32_t b[2] = { h & t->nbkt_mask, alt_bucket(h, t->nbkt_mask) };

	for (int k = 0; k < 2; k++) {
		const struct orc_bucket *bk = &t->bkt[b[k]];
		for (int s = 0; s < ORC_BKT; s++)
			if (bk->uid[s] >= 0 && bk->sig[s] == h && bk->ip[s] == ip)
				return bk->uid[s];
	}
	return -1;
}

static int iptab_add(struct orc_tables *t, uint32_t ip, int uid)
{
	uint32_t h = orc_jhash(&ip, 4);
	uint32_t b[2] = { h & t->nbkt_mask, alt_bucket(h, t->nbkt_mask) };

	for (int k = 0; k < 2; k++) {
		struct orc_bucket *bk = &t->bkt[b[k]];
		for (int s = 0; s < ORC_BKT; s++) {
			if (bk->uid[s] < 0) {
				bk->uid[s] = uid;
				bk->sig[s] = h;
				bk->ip[s] = ip;
				return 0;
			}
		}
	}
	return -ENOSPC;
}

static void iptab_del(struct orc_tables *t, uint32_t ip)
{
	uint32_t h = orc_jhash(&ip, 4);
	uint32_t b[2] = { h & t->nbkt_mask, alt_bucket(h, t->nbkt_mask) };

	for (int k = 0; k < 2; k++) {
		struct orc_bucket *bk = &t->bkt[b[k]];
		for (int s = 0; s < ORC_BKT; s++)
			if (bk->uid[s] >= 0 && bk->ip[s] == ip)
				bk->uid[s] = -1;
	}
}

int orc_runtime_set(struct orc_tables *t, uint16_t uniqid, uint32_t ip,
                    uint16_t thread_count, uint16_t active,
                    const uint16_t *flow_tbl)
{
	struct orc_runtime *r;
	int owner;

	if (uniqid >= t->max_runtimes || thread_count == 0 ||
	    thread_count > GCL_NCPU || active > thread_count)
		return -EINVAL;
	if (active) {
		for (int i = 0; i < thread_count; i++)
			if (flow_tbl[i] >= thread_count)
				return -EINVAL;
	}
	owner = iptab_lookup(t, ip);
	if (owner >= 0 && owner != uniqid)
		return -EEXIST; /* dp_clients.c:174-179 */
	r = &t->rt[uniqid];
	if (r->present && r->ip != ip)
		iptab_del(t, r->ip);
	if (owner < 0 || (r->present && r->ip != ip)) {
		int ret = iptab_add(t, ip, uniqid);
		if (ret)
			return ret;
	}
	if (!r->present)
		t->trans_seed[uniqid] = 0;
	r->present = 1;
	r->ip = ip;
	r->thread_count = thread_count;
	r->active = active;
	if (active)
		memcpy(r->flow_tbl, flow_tbl, thread_count * sizeof(uint16_t));
	return 0;
}

int orc_runtime_set_trans_seed(struct orc_tables *t, uint16_t uniqid, uint32_t seed)
{
	if (uniqid >= t->max_runtimes || !t->rt[uniqid].present)
		return -ENOENT;
	t->trans_seed[uniqid] = seed;
	return 0;
}

int orc_runtime_del(struct orc_tables *t, uint16_t uniqid)
{
	if (uniqid >= t->max_runtimes || !t->rt[uniqid].present)
		return -ENOENT;
	iptab_del(t, t->rt[uniqid].ip);
	memset(&t->rt[uniqid], 0, sizeof(t->rt[uniqid]));
	t->trans_seed[uniqid] = 0;
	return 0;
}

/* ------------------------------------------------------------------------
 * Classifier.
 */
struct pkt_view {
	const uint8_t *base;  /* frame start, or NULL if out of range */
	uint64_t off;
	uint64_t frames_len;
	const uint8_t *frames;
};

/* byte k of the frame; bytes past frames_len read as 0 */
static inline uint8_t fb(const struct pkt_view *pv, uint64_t k)
{
	/* no off + k: an offset near 2^64 must read 0, not wrap into the buffer */
	return pv->off < pv->frames_len && k < pv->frames_len - pv->off ? pv->frames[pv->off + k] : 0;
}

static inline uint16_t fbe16(const struct pkt_view *pv, uint64_t k)
{
	return (uint16_t)(fb(pv, k) << 8 | fb(pv, k + 1));
}

static inline uint32_t fbe32(const struct pkt_view *pv, uint64_t k)
{
	return (uint32_t)fbe16(pv, k) << 16 | fbe16(pv, k + 2);
}

/* The build-defined flow hash of the computed modes (gclassify.h). */
static uint32_t flow_hash(const struct orc_tables *t, const struct pkt_view *pv)
{
	uint8_t key[13];
	uint32_t saddr, daddr;
	uint16_t sport, dport, frag;
	uint8_t ihl, proto;

	if (fbe16(pv, 12) != GCL_ETHTYPE_IP)
		return 0;
	ihl = fb(pv, 14) & 0xF;
	frag = fbe16(pv, 20);
	proto = fb(pv, 23);
	if (ihl < 5 || (frag & 0x3FFF) || (proto != 6 && proto != 17))
		return 0;
	saddr = fbe32(pv, 26);
	daddr = fbe32(pv, 30);
	sport = fbe16(pv, 14 + 4u * ihl);
	dport = fbe16(pv, 16 + 4u * ihl);
	if (t->hash_mode == GCL_HASH_TOEPLITZ)
		return orc_do_toeplitz(t->rss_key, saddr, daddr, sport, dport);
	memcpy(key, &saddr, 4);      /* host-order (LE) fields */
	memcpy(key + 4, &daddr, 4);
	memcpy(key + 8, &dport, 2);
	memcpy(key + 10, &sport, 2);
	key[12] = proto;
	return orc_jhash(key, 13);
}

/*
 * rx_one_pkt, iokernel/rx.c:116-233, with rx_send_pkt_to_runtime (:76-92)
 * and rx_send_to_runtime (:50-73) reduced to the steering decision.
 */
/*
 * Transport demux hashes the destination runtime computes in trans_lookup
 * (runtime/net/transport.c:29-42, :366-375) for the frames net_rx_one hands
 * to net_rx_trans: IPv4, ip_hdr_supported as written (core.c:203-209, IP_MF
 * tested on the network-order field), TCP or UDP.  L4 right after the
 * 20-byte header (mbuf_pull_hdr of struct ip_hdr, core.c:272).
 */
static int orc_trans(const struct orc_tables *t, const struct pkt_view *pv, int p,
                     struct gcl_trans *tr)
{
	uint8_t vihl = fb(pv, 14), proto = fb(pv, 23);
	uint16_t off_raw = (uint16_t)(fb(pv, 20) | fb(pv, 21) << 8);
	uint32_t seed = t->trans_seed[p];
	uint64_t l, r;

	if (fbe16(pv, 12) != GCL_ETHTYPE_IP || (vihl >> 4) != 4 || (vihl & 0xF) != 5 ||
	    (off_raw & 0x2000) || (proto != 6 && proto != 17))
		return 0;
	l = (uint64_t)fbe32(pv, 30) | (uint64_t)fbe16(pv, 36) << 32;
	r = (uint64_t)fbe32(pv, 26) | (uint64_t)fbe16(pv, 34) << 32 | (uint64_t)proto << 48;
	tr->h5 = orc_crc32c_u64(orc_crc32c_u64(seed, l), r);
	tr->h3 = orc_crc32c_u64(seed, l | (uint64_t)proto << 48);
	return 1;
}

static void orc_rx_one_pkt(const struct orc_tables *t, const struct gcl_batch *b,
                           uint64_t i, struct gcl_verdict *v, uint64_t *counts,
                           uint64_t *stats, struct gcl_trans *tr)
{
	struct pkt_view pv;
	uint8_t flags = b->olflags ? b->olflags[i] : t->default_olflags;
	uint32_t hash, dst_ip = 0;
	uint16_t et;
	int p = -1, fdir = 0;

	pv.frames = b->frames;
	pv.frames_len = b->frames_len;
	pv.off = b->offs ? b->offs[i] : i * b->stride;

	if (t->hash_mode == GCL_HASH_NIC)
		hash = b->rss ? b->rss[i] : 0;
	else
		hash = flow_hash(t, &pv);
	if (t->flags & GCL_CFG_HASH16)
		hash &= 0xFFFF;
	v->hash = hash;
	v->uniqid = GCL_NO_RUNTIME;
	v->thread = GCL_NO_THREAD;
	if (tr)
		tr->h5 = tr->h3 = 0;

	/* rx_loopback, rx.c:249-262: a tx dst_ip hint found in ip_to_proc sets
	 * RTE_MBUF_F_RX_FDIR_ID with hash.fdir.hi = p->uniqid */
	int hint_p = -1;
	if (b->dst_hint && b->dst_hint[i]) {
		hint_p = iptab_lookup(t, b->dst_hint[i]);
		if (hint_p >= 0)
			flags |= GCL_F_FDIR_ID;
	}

	/* hardware flow tag, rx.c:131-146 */
	if (flags & GCL_F_FDIR_ID) {
		uint32_t mark = hint_p >= 0 ? (uint32_t)hint_p : (b->fdir_hi ? b->fdir_hi[i] : 0);
		stats[GCL_RX_FLOW_TAG_MATCH]++;
		if (mark < t->max_runtimes && t->rt[mark].present) {
			p = (int)mark;
			fdir = GCL_ACT_F_FDIR;
			goto deliver;
		}
		/* NULL proc: fall through to the header parse */
	}

	et = fbe16(&pv, 12); /* rx.c:154 */
	if (et == GCL_ETHTYPE_IP) {
		dst_ip = fbe32(&pv, 30); /* rx.c:157-159: fixed offset, no IHL */
		if (!(flags & GCL_F_RSS_HASH))
			stats[GCL_RX_HASH_MISSING]++;
	} else if (et == GCL_ETHTYPE_ARP) {
		dst_ip = fbe32(&pv, 38); /* arp_tip, rx.c:165-167 */
		if ((t->flags & GCL_CFG_AZURE_ARP) &&
		    fbe16(&pv, 20) == GCL_ARP_OP_REPLY) {
			v->action = GCL_ACT_BROADCAST; /* rx.c:171-190 */
			return;
		}
	} else {
		v->action = GCL_ACT_DROP_ETHERTYPE; /* rx.c:191-194 */
		stats[GCL_RX_UNHANDLED]++;
		return;
	}

	p = iptab_lookup(t, dst_ip); /* rx.c:197 */
	if (p < 0) {
		if ((t->flags & GCL_CFG_AZURE_ARP) && et == GCL_ETHTYPE_ARP &&
		    fbe16(&pv, 20) == GCL_ARP_OP_REQUEST) {
			v->action = GCL_ACT_ARP_RESPOND; /* rx.c:200-203 */
			return;
		}
		stats[GCL_RX_UNREGISTERED_MAC]++; /* rx.c:205 */
		stats[GCL_RX_UNHANDLED]++;        /* rx.c:232 */
		v->action = GCL_ACT_DROP_UNREG;
		return;
	}

deliver:
	v->uniqid = (uint16_t)p;
	counts[p]++;
	/* rx_send_to_runtime's flow_tbl slot, hash % thread_count (rx.c:57, :68);
	 * flow_tbl[slot] is read by the post-pass at delivery time */
	v->thread = (uint8_t)(hash % t->rt[p].thread_count);
	if (t->rt[p].active > 0) /* rx.c:55-59 */
		v->action = (uint8_t)(GCL_ACT_DELIVER | fdir);
	else
		v->action = (uint8_t)(GCL_ACT_WAKE | fdir); /* rx.c:62-72 */
	if (tr && (t->flags & GCL_CFG_TRANS_HASH) && orc_trans(t, &pv, p, tr))
		v->action |= GCL_ACT_F_TRANS;
}

/*
 * rx_one_pkt as rx.c:116-233 writes it, for the CPU BASELINE only: header
 * fields loaded straight through header structs at the frame pointer
 * (rte_pktmbuf_mtod + ether_type / iphdr->dst_addr / arp_tip, rx.c:127-167),
 * no per-byte bounds test, and in GCL_HASH_NIC mode the NIC's hash.rss
 * (rx.c:83) -- what the dataplane core really does per packet.  The caller
 * guarantees every frame's first 42 bytes (54 with L4 ports) lie inside the
 * buffer, as an mbuf's data does.  Same verdicts as orc_rx_one_pkt for such
 * batches without loopback hints (tests/test_oracle_scenarios.py).
 */
struct rb_eth { uint8_t dst[6], src[6]; uint16_t type; } __attribute__((packed));
struct rb_ip {
	uint8_t vihl, tos;
	uint16_t len, id, off;
	uint8_t ttl, proto;
	uint16_t csum;
	uint32_t saddr, daddr;
} __attribute__((packed));
struct rb_arp {
	uint16_t htype, ptype;
	uint8_t hlen, plen;
	uint16_t op;
	uint8_t sha[6];
	uint32_t sip;
	uint8_t tha[6];
	uint32_t tip;
} __attribute__((packed));

static inline uint32_t rb_flow_hash(const struct orc_tables *t, const uint8_t *f)
{
	const struct rb_ip *ip = (const struct rb_ip *)(f + sizeof(struct rb_eth));
	const unsigned ihl = ip->vihl & 0xF;
	uint8_t key[13];
	uint32_t saddr, daddr;
	uint16_t sport, dport, ports[2];

	if (__builtin_bswap16(((const struct rb_eth *)f)->type) != GCL_ETHTYPE_IP || ihl < 5 ||
	    (__builtin_bswap16(ip->off) & 0x3FFF) || (ip->proto != 6 && ip->proto != 17))
		return 0;
	memcpy(ports, f + sizeof(struct rb_eth) + 4 * ihl, 4);
	saddr = __builtin_bswap32(ip->saddr);
	daddr = __builtin_bswap32(ip->daddr);
	sport = __builtin_bswap16(ports[0]);
	dport = __builtin_bswap16(ports[1]);
	if (t->hash_mode == GCL_HASH_TOEPLITZ)
		return orc_do_toeplitz(t->rss_key, saddr, daddr, sport, dport);
	memcpy(key, &saddr, 4);
	memcpy(key + 4, &daddr, 4);
	memcpy(key + 8, &dport, 2);
	memcpy(key + 10, &sport, 2);
	key[12] = ip->proto;
	return orc_jhash(key, 13);
}

static inline void rx_one_pkt_direct(const struct orc_tables *t, const struct gcl_batch *b,
                                     uint64_t i, struct gcl_verdict *v, uint64_t *counts,
                                     uint64_t *stats)
{
	const uint8_t *f = b->frames + (b->offs ? b->offs[i] : i * b->stride);
	const struct rb_eth *eh = (const struct rb_eth *)f;
	const uint8_t flags = b->olflags ? b->olflags[i] : t->default_olflags;
	uint32_t hash, dst_ip;
	uint16_t et;
	int p;

	hash = t->hash_mode == GCL_HASH_NIC ? (b->rss ? b->rss[i] : 0) : rb_flow_hash(t, f);
	if (t->flags & GCL_CFG_HASH16)
		hash &= 0xFFFF;
	v->hash = hash;
	v->uniqid = GCL_NO_RUNTIME;
	v->thread = GCL_NO_THREAD;
	if (flags & GCL_F_FDIR_ID) { /* rx.c:131-146 */
		const uint32_t mark = b->fdir_hi ? b->fdir_hi[i] : 0;
		stats[GCL_RX_FLOW_TAG_MATCH]++;
		if (mark < t->max_runtimes && t->rt[mark].present) {
			p = (int)mark;
			goto deliver_fdir;
		}
	}
	et = __builtin_bswap16(eh->type); /* rx.c:154 */
	if (__builtin_expect(et == GCL_ETHTYPE_IP, 1)) {
		const struct rb_ip *ip = (const struct rb_ip *)(f + sizeof(*eh));
		dst_ip = __builtin_bswap32(ip->daddr); /* rx.c:157-159 */
		if (!(flags & GCL_F_RSS_HASH))
			stats[GCL_RX_HASH_MISSING]++;
	} else if (et == GCL_ETHTYPE_ARP) {
		const struct rb_arp *ah = (const struct rb_arp *)(f + sizeof(*eh));
		dst_ip = __builtin_bswap32(ah->tip); /* rx.c:165-167 */
		if ((t->flags & GCL_CFG_AZURE_ARP) && __builtin_bswap16(ah->op) == GCL_ARP_OP_REPLY) {
			v->action = GCL_ACT_BROADCAST;
			return;
		}
	} else {
		v->action = GCL_ACT_DROP_ETHERTYPE; /* rx.c:191-194 */
		stats[GCL_RX_UNHANDLED]++;
		return;
	}
	p = iptab_lookup(t, dst_ip); /* rx.c:197 */
	if (__builtin_expect(p < 0, 0)) {
		if ((t->flags & GCL_CFG_AZURE_ARP) && et == GCL_ETHTYPE_ARP &&
		    __builtin_bswap16(((const struct rb_arp *)(f + sizeof(*eh)))->op) ==
		            GCL_ARP_OP_REQUEST) {
			v->action = GCL_ACT_ARP_RESPOND;
			return;
		}
		stats[GCL_RX_UNREGISTERED_MAC]++;
		stats[GCL_RX_UNHANDLED]++;
		v->action = GCL_ACT_DROP_UNREG;
		return;
	}
	v->uniqid = (uint16_t)p;
	counts[p]++;
	v->thread = (uint8_t)(hash % t->rt[p].thread_count); /* the flow_tbl slot */
	v->action = t->rt[p].active > 0 ? GCL_ACT_DELIVER : GCL_ACT_WAKE; /* rx.c:55-72 */
	return;
deliver_fdir:
	v->uniqid = (uint16_t)p;
	counts[p]++;
	v->thread = (uint8_t)(hash % t->rt[p].thread_count);
	v->action = (t->rt[p].active > 0 ? GCL_ACT_DELIVER : GCL_ACT_WAKE) | GCL_ACT_F_FDIR;
}

#define RX_PREFETCH_STRIDE 2 /* rx.c:22 */

static void classify_range_direct(const struct orc_tables *t, const struct gcl_batch *b,
                                  uint64_t lo, uint64_t hi, struct gcl_verdict *v,
                                  uint64_t *counts, uint64_t *stats)
{
	/* rx_burst, rx.c:270-290, over rx_one_pkt_direct */
	for (uint64_t s = lo; s < hi; s += GCL_RX_BURST_SIZE) {
		uint64_t nb = hi - s < GCL_RX_BURST_SIZE ? hi - s : GCL_RX_BURST_SIZE;
		stats[GCL_RX_PULLED] += nb;
		for (uint64_t i = 0; i < nb; i++) {
			if (i + RX_PREFETCH_STRIDE < nb) {
				uint64_t j = s + i + RX_PREFETCH_STRIDE;
				__builtin_prefetch(b->frames + (b->offs ? b->offs[j] : j * b->stride));
			}
			rx_one_pkt_direct(t, b, s + i, &v[s + i - lo], counts, stats);
		}
	}
}

static void classify_range(const struct orc_tables *t, const struct gcl_batch *b,
                           uint64_t lo, uint64_t hi, struct gcl_verdict *v,
                           uint64_t *counts, uint64_t *stats, struct gcl_trans *tr)
{
	/* rx_burst, rx.c:270-290: bursts of IOKERNEL_RX_BURST_SIZE */
	for (uint64_t s = lo; s < hi; s += GCL_RX_BURST_SIZE) {
		uint64_t nb = hi - s < GCL_RX_BURST_SIZE ? hi - s : GCL_RX_BURST_SIZE;
		stats[GCL_RX_PULLED] += nb;
		for (uint64_t i = 0; i < nb; i++) {
			if (i + RX_PREFETCH_STRIDE < nb) {
				uint64_t j = s + i + RX_PREFETCH_STRIDE;
				uint64_t off = b->offs ? b->offs[j] : j * b->stride;
				if (off < b->frames_len)
					__builtin_prefetch(b->frames + off);
			}
			orc_rx_one_pkt(t, b, s + i, &v[s + i - lo], counts, stats,
			               tr ? &tr[s + i - lo] : NULL);
		}
	}
}

void orc_classify(const struct orc_tables *t, const struct gcl_batch *b,
                  struct gcl_verdict *v, uint64_t *counts, uint64_t *stats)
{
	classify_range(t, b, 0, b->n, v, counts, stats, NULL);
}

void orc_classify_direct(const struct orc_tables *t, const struct gcl_batch *b,
                         struct gcl_verdict *v, uint64_t *counts, uint64_t *stats)
{
	classify_range_direct(t, b, 0, b->n, v, counts, stats);
}

void orc_classify_ex(const struct orc_tables *t, const struct gcl_batch *b,
                     struct gcl_verdict *v, uint64_t *counts, uint64_t *stats,
                     struct gcl_trans *tr)
{
	classify_range(t, b, 0, b->n, v, counts, stats, tr);
}

/* lrpc ring, inc/base/lrpc.h:15-63 (16-B messages, parity in bit 63) */
struct orc_lrpc {
	uint32_t send_head, send_tail, size;
	uint64_t *tbl; /* 2 words per message */
};

static int lrpc_send(struct orc_lrpc *c, uint64_t cmd, uint64_t payload)
{
	uint64_t *dst;

	if (c->send_head - c->send_tail >= c->size) {
		/* __lrpc_send's refresh from recv_head_wb (base/lrpc.c:16-19):
		 * the emulated runtime consumes instantly, so its head is ours */
		c->send_tail = c->send_head;
		if (c->send_head - c->send_tail >= c->size)
			return 0; /* ring full: RX_UNICAST_FAIL */
	}
	dst = &c->tbl[2 * (c->send_head & (c->size - 1))];
	cmd |= (c->send_head++ & c->size) ? 0 : (1ull << 63);
	dst[1] = payload;
	__atomic_store_n(&dst[0], cmd, __ATOMIC_RELEASE);
	return 1;
}

struct lrpc_set {
	struct orc_lrpc *rings; /* [max_runtimes * GCL_NCPU_USED] lazily allocated */
	uint32_t stride;
};

#define LRPC_DEPTH 4096 /* runtime/ioqueues.c:31-40 */

static struct orc_lrpc *ring_of(struct lrpc_set *s, uint32_t p, uint32_t th)
{
	struct orc_lrpc *r = &s->rings[p * s->stride + th];
	if (!r->tbl) {
		r->tbl = calloc(2 * LRPC_DEPTH, sizeof(uint64_t));
		r->size = LRPC_DEPTH;
	}
	return r;
}

/* rx_burst's loop with the post-pass of every delivered packet: @post 2
 * rx_make_cmd + flow_tbl[slot] + lrpc_send (rx.c:76-92), 1 all but the ring
 * write (ORC_BENCH_NOSEND), 0 none (the direct CPU baseline's classify-only
 * cell).  Not inlined, so the classify-only and lrpc cells time one loop
 * that differs only by @post: inlined separately, the two loops' code
 * differed enough that on the mixed stream the one with the ring writes ran
 * 3 % faster (gpurun_out/r05i_bench_detail.json) */
__attribute__((noinline)) static void classify_range_lrpc(const struct orc_tables *t, const struct gcl_batch *b,
                                                          uint64_t lo, uint64_t hi, struct gcl_verdict *v,
                                                          uint64_t *counts, uint64_t *stats,
                                                          struct lrpc_set *rs, int direct, int post)
{
	uint64_t sink = 0;
	for (uint64_t s = lo; s < hi; s += GCL_RX_BURST_SIZE) {
		uint64_t nb = hi - s < GCL_RX_BURST_SIZE ? hi - s : GCL_RX_BURST_SIZE;
		stats[GCL_RX_PULLED] += nb;
		for (uint64_t i = 0; i < nb; i++) {
			uint64_t k = s + i;
			struct gcl_verdict *vk = &v[k - lo];
			if (i + RX_PREFETCH_STRIDE < nb) {
				uint64_t j = k + RX_PREFETCH_STRIDE;
				uint64_t off = b->offs ? b->offs[j] : j * b->stride;
				if (off < b->frames_len)
					__builtin_prefetch(b->frames + off);
			}
			if (direct)
				rx_one_pkt_direct(t, b, k, vk, counts, stats);
			else
				orc_rx_one_pkt(t, b, k, vk, counts, stats, NULL);
			if (post && (vk->action & GCL_ACT_MASK) == GCL_ACT_DELIVER) {
				/* rx_make_cmd, rx.c:24-38 */
				uint8_t fl = b->olflags ? b->olflags[k] : t->default_olflags;
				uint64_t len = b->pkt_len ? b->pkt_len[k] : b->stride;
				uint64_t csum = (fl & GCL_F_IP_CKSUM_MASK) == GCL_F_IP_CKSUM_GOOD;
				uint64_t cmd = 0 | (len & 0xFFFF) << 16 | csum << 48;
				uint64_t off = b->offs ? b->offs[k] : k * b->stride;
				/* rx_send_to_runtime: flow_tbl[slot] at send time (rx.c:57) */
				const uint32_t th = t->rt[vk->uniqid].flow_tbl[vk->thread];
				if (post == 1) { /* ORC_BENCH_NOSEND: everything but the ring write */
					sink += cmd ^ off ^ th;
				} else if (!lrpc_send(ring_of(rs, vk->uniqid, th), cmd, off)) {
					stats[GCL_RX_UNICAST_FAIL]++;
					stats[GCL_RX_UNHANDLED]++;
				}
			}
		}
		/* the runtimes drain their rings: seen lazily, when a ring looks
		 * full (lrpc_send), as the GPU pipeline's rings (tools/rxpipe.cpp) */
	}
	if (sink == 0x9E3779B97F4A7C15ull) /* keeps the no-send loop's work live */
		stats[GCL_RX_UNICAST_FAIL] += 0;
	__asm__ volatile("" : : "r"(sink));
}

static uint32_t max_threads(const struct orc_tables *t)
{
	uint32_t m = 1;
	for (uint32_t i = 0; i < t->max_runtimes; i++)
		if (t->rt[i].present && t->rt[i].thread_count > m)
			m = t->rt[i].thread_count;
	return m;
}

static void lrpc_set_init(struct lrpc_set *s, const struct orc_tables *t)
{
	s->stride = max_threads(t);
	s->rings = calloc((size_t)t->max_runtimes * s->stride, sizeof(*s->rings));
}

static void lrpc_set_free(struct lrpc_set *s, const struct orc_tables *t)
{
	for (size_t i = 0; i < (size_t)t->max_runtimes * s->stride; i++)
		free(s->rings[i].tbl);
	free(s->rings);
}

void orc_classify_lrpc(const struct orc_tables *t, const struct gcl_batch *b,
                       struct gcl_verdict *v, uint64_t *counts, uint64_t *stats)
{
	struct lrpc_set rs;
	lrpc_set_init(&rs, t);
	classify_range_lrpc(t, b, 0, b->n, v, counts, stats, &rs, 0, 2);
	lrpc_set_free(&rs, t);
}

struct orc_dataplane {
	const struct orc_tables *t;
	struct lrpc_set rs;
};

struct orc_dataplane *orc_dataplane_new(const struct orc_tables *t)
{
	struct orc_dataplane *d = calloc(1, sizeof(*d));
	if (!d)
		return NULL;
	d->t = t;
	lrpc_set_init(&d->rs, t);
	return d;
}

void orc_dataplane_free(struct orc_dataplane *d)
{
	if (!d)
		return;
	lrpc_set_free(&d->rs, d->t);
	free(d);
}

void orc_dataplane_burst(struct orc_dataplane *d, const struct gcl_batch *b, struct gcl_verdict *v,
                         uint64_t *counts, uint64_t *stats, int send)
{
	classify_range_lrpc(d->t, b, 0, b->n, v, counts, stats, &d->rs, 1, send ? 2 : 0);
}

/* ------------------------------------------------------------------------
 * CPU baseline timer.
 */
struct bench_arg {
	const struct orc_tables *t;
	const struct gcl_batch *b;
	uint64_t lo, hi;
	int passes, with_lrpc, direct, send;
	int cpu; /* pinned to this CPU before the clock starts (-1: not pinned) */
	pthread_barrier_t *bar;
};

static void *bench_thread(void *arg)
{
	struct bench_arg *a = arg;
	uint64_t n = a->hi - a->lo;
	struct gcl_verdict *v = malloc((n ? n : 1) * sizeof(*v));
	uint64_t *counts = calloc(a->t->max_runtimes, sizeof(uint64_t));
	uint64_t stats[GCL_NR_STATS] = { 0 };
	struct lrpc_set rs = { 0 };

	if (a->cpu >= 0) { /* as the iokernel pins its dataplane lcore, dpdk.c:276-280 */
		cpu_set_t one;
		CPU_ZERO(&one);
		CPU_SET(a->cpu, &one);
		(void)pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
	}
	if (a->with_lrpc)
		lrpc_set_init(&rs, a->t);
	/* one untimed pass on this thread's own core first: the verdict buffer
	 * and the rings touched, the shard's frame lines pulled out of whichever
	 * cache the previous run left them in -- the steady state of a
	 * dataplane core that has been polling all along */
	for (int p = -1; p < a->passes; p++) {
		if (p == 0)
			pthread_barrier_wait(a->bar);
		if (a->with_lrpc || a->direct)
			classify_range_lrpc(a->t, a->b, a->lo, a->hi, v, counts, stats, &rs, a->direct,
			                    a->with_lrpc ? (a->send ? 2 : 1) : 0);
		else
			classify_range(a->t, a->b, a->lo, a->hi, v, counts, stats, NULL);
	}
	if (a->passes < 1)
		pthread_barrier_wait(a->bar);
	pthread_barrier_wait(a->bar);
	if (a->with_lrpc)
		lrpc_set_free(&rs, a->t);
	free(v);
	free(counts);
	return NULL;
}

double orc_bench(const struct orc_tables *t, const struct gcl_batch *b,
                 int threads, int passes, int with_lrpc)
{
	return orc_bench_ex(t, b, threads, passes, with_lrpc ? ORC_BENCH_LRPC : 0);
}

double orc_bench_ex(const struct orc_tables *t, const struct gcl_batch *b,
                    int threads, int passes, unsigned int flags)
{
	return orc_bench_pinned(t, b, threads, passes, flags, NULL);
}

double orc_bench_pinned(const struct orc_tables *t, const struct gcl_batch *b,
                        int threads, int passes, unsigned int flags, const int *cpus)
{
	pthread_t tid[256];
	struct bench_arg arg[256];
	pthread_barrier_t bar;
	struct timespec t0, t1;

	if (threads < 1)
		threads = 1;
	if (threads > 256)
		threads = 256;
	pthread_barrier_init(&bar, NULL, (unsigned)threads + 1);
	for (int i = 0; i < threads; i++) {
		arg[i].t = t;
		arg[i].b = b;
		arg[i].lo = b->n * (uint64_t)i / (uint64_t)threads;
		arg[i].hi = b->n * (uint64_t)(i + 1) / (uint64_t)threads;
		arg[i].passes = passes;
		arg[i].with_lrpc = !!(flags & (ORC_BENCH_LRPC | ORC_BENCH_NOSEND));
		arg[i].send = !(flags & ORC_BENCH_NOSEND);
		arg[i].direct = !!(flags & ORC_BENCH_DIRECT);
		arg[i].cpu = cpus ? cpus[i] : -1;
		arg[i].bar = &bar;
		pthread_create(&tid[i], NULL, bench_thread, &arg[i]);
	}
	pthread_barrier_wait(&bar);
	clock_gettime(CLOCK_MONOTONIC, &t0);
	pthread_barrier_wait(&bar);
	clock_gettime(CLOCK_MONOTONIC, &t1);
	for (int i = 0; i < threads; i++)
		pthread_join(tid[i], NULL);
	pthread_barrier_destroy(&bar);
	return (double)(t1.tv_sec - t0.tv_sec) + (double)(t1.tv_nsec - t0.tv_nsec) * 1e-9;
}

/* ------------------------------------------------------------------------
 * Synthetic generator (same streams as the device generator).
 */
static inline uint64_t mix64(uint64_t z)
{
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

/* k-th random word of global packet g: splitmix64 at position 8g+k */
static inline uint64_t rw(uint64_t seed, uint64_t g, uint64_t k)
{
	return mix64(seed + (g * 8 + k + 1) * 0x9E3779B97F4A7C15ull);
}

uint32_t orc_runtime_ip(uint32_t r)
{
	return 0x0A000000u + r + 1; /* 10.0.0.0 + r + 1 */
}

int orc_zipf_cdf(uint32_t nflows, double s, uint64_t *cdf)
{
	double h = 0.0, acc = 0.0;

	if (nflows == 0)
		return -EINVAL;
	for (uint32_t k = 0; k < nflows; k++)
		h += pow((double)k + 1.0, -s);
	for (uint32_t k = 0; k < nflows; k++) {
		double x;
		acc += pow((double)k + 1.0, -s);
		x = ldexp(acc / h, 64);
		cdf[k] = x >= 18446744073709551615.0 ? UINT64_MAX : (uint64_t)x;
	}
	cdf[nflows - 1] = UINT64_MAX;
	return 0;
}

static uint32_t zipf_pick(const uint64_t *cdf, uint32_t nflows, uint64_t u)
{
	uint32_t lo = 0, hi = nflows - 1;
	while (lo < hi) { /* first k with u < cdf[k] */
		uint32_t mid = lo + (hi - lo) / 2;
		if (u < cdf[mid])
			hi = mid;
		else
			lo = mid + 1;
	}
	return lo;
}

static void put16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static void put32(uint8_t *p, uint32_t v) { put16(p, (uint16_t)(v >> 16)); put16(p + 2, (uint16_t)v); }

static void ip_csum(uint8_t *ip)
{
	uint32_t s = 0;
	ip[10] = ip[11] = 0;
	for (int i = 0; i < 20; i += 2)
		s += (uint32_t)ip[i] << 8 | ip[i + 1];
	while (s >> 16)
		s = (s & 0xFFFF) + (s >> 16);
	put16(ip + 10, (uint16_t)~s);
}

static void eth(uint8_t *f, uint64_t srcbits, uint16_t et)
{
	static const uint8_t dmac[6] = { 0x02, 0x00, 0x00, 0x00, 0x00, 0x01 };
	memcpy(f, dmac, 6);
	f[6] = 0x02;
	f[7] = 0x00;
	put32(f + 8, (uint32_t)srcbits);
	put16(f + 12, et);
}

static void ipv4(uint8_t *ip, uint16_t totlen, uint16_t id, uint8_t proto,
                 uint32_t saddr, uint32_t daddr)
{
	ip[0] = 0x45;
	ip[1] = 0;
	put16(ip + 2, totlen);
	put16(ip + 4, id);
	put16(ip + 6, 0x4000); /* DF */
	ip[8] = 64;
	ip[9] = proto;
	put32(ip + 12, saddr);
	put32(ip + 16, daddr);
	ip_csum(ip);
}

static uint64_t global_index(const struct gcl_gen_params *p, uint64_t j)
{
	if (!p->shard_block || p->world <= 1)
		return j;
	return ((j / p->shard_block) * p->world + p->rank) * p->shard_block +
	       j % p->shard_block;
}

int orc_generate(const struct gcl_gen_params *p, const uint64_t *zipf_cdf,
                 uint8_t *frames, uint8_t *olflags, uint32_t *rss)
{
	if (p->stride < 64 || p->nruntimes == 0)
		return -EINVAL;
	for (uint64_t j = 0; j < p->n; j++) {
		uint64_t g = global_index(p, j);
		uint8_t *f = frames + j * p->stride;
		uint64_t r0 = rw(p->seed, g, 0), r1 = rw(p->seed, g, 1);
		uint8_t fl = GCL_F_RSS_HASH | GCL_F_IP_CKSUM_GOOD;
		uint16_t len = 64;

		memset(f, 0, 64);
		if (p->workload == GCL_WL_UDP64) {
			uint32_t rt = (uint32_t)(((uint64_t)(uint32_t)r1 * p->nruntimes) >> 32);
			eth(f, r1 >> 32, GCL_ETHTYPE_IP);
			ipv4(f + 14, 50, (uint16_t)(r1 >> 16), 17, (uint32_t)r0,
			     orc_runtime_ip(rt));
			put16(f + 34, (uint16_t)(r0 >> 32));
			put16(f + 36, (uint16_t)(r0 >> 48));
			put16(f + 38, 30);
		} else if (p->workload == GCL_WL_TCP1500_ZIPF) {
			uint32_t flow, rt;
			uint64_t fr;
			if (!zipf_cdf || !p->nflows)
				return -EINVAL;
			flow = zipf_pick(zipf_cdf, p->nflows, r0);
			fr = rw(p->seed ^ 0xF10F10F10F10F10Full, flow, 0);
			rt = flow % p->nruntimes;
			eth(f, fr >> 16, GCL_ETHTYPE_IP);
			ipv4(f + 14, 1486, (uint16_t)r1, 6, (uint32_t)fr, orc_runtime_ip(rt));
			put16(f + 34, (uint16_t)(fr >> 32));
			put16(f + 36, (uint16_t)(fr >> 48));
			put32(f + 38, (uint32_t)(r1 >> 32)); /* seq */
			f[46] = 0x50;                         /* data offset 5 */
			f[47] = 0x10;                         /* ACK */
			put16(f + 48, 0xFFFF);                /* window */
			len = 1500;
		} else if (p->workload == GCL_WL_MIXED) {
			uint64_t r2 = rw(p->seed, g, 2);
			uint32_t kind = (uint32_t)r0 % 100;
			uint32_t rt = (uint32_t)(((uint64_t)(uint32_t)r1 * p->nruntimes) >> 32);
			int unreg = (uint32_t)(r0 >> 40) % 20 == 0;
			uint32_t dst = unreg ? 0xC0A80000u | (uint32_t)(r1 >> 48) : orc_runtime_ip(rt);
			if (kind < 70) {
				len = (uint16_t)(64 + (uint32_t)(r1 >> 32) % (9014 - 64 + 1));
				uint8_t proto = (r0 >> 32) & 1 ? 6 : 17;
				eth(f, r2 >> 8, GCL_ETHTYPE_IP);
				ipv4(f + 14, (uint16_t)(len - 14), (uint16_t)r2, proto,
				     (uint32_t)r2, dst);
				put16(f + 34, (uint16_t)(r2 >> 32));
				put16(f + 36, (uint16_t)(r2 >> 48));
			} else if (kind < 90) {
				eth(f, r2 >> 8, GCL_ETHTYPE_IPV6);
				f[14] = 0x60;
				put16(f + 18, (uint16_t)(r1 >> 32) & 0x1FFF);
				f[20] = 17;
				f[21] = 64;
				put32(f + 22, (uint32_t)r2);
				put32(f + 38, dst);
				fl = 0;
				len = (uint16_t)(54 + ((uint32_t)(r1 >> 32) & 0x1FFF));
				len = len < 60 ? 60 : len;
			} else {
				unreg = (uint32_t)(r0 >> 40) % 10 == 0;
				dst = unreg ? 0xC0A80000u | (uint32_t)(r1 >> 48) : orc_runtime_ip(rt);
				eth(f, r2 >> 8, GCL_ETHTYPE_ARP);
				put16(f + 14, 1);      /* htype ether */
				put16(f + 16, 0x0800); /* ptype */
				f[18] = 6;
				f[19] = 4;
				put16(f + 20, (r0 >> 33) & 1 ? GCL_ARP_OP_REPLY : GCL_ARP_OP_REQUEST);
				put32(f + 24, (uint32_t)(r2 >> 16)); /* sha (part) */
				put32(f + 28, (uint32_t)r2);         /* sip */
				put32(f + 38, dst);                  /* tip */
				fl = 0;
				len = 60;
			}
		} else {
			return -EINVAL;
		}
		if (olflags)
			olflags[j] = fl;
		if (rss)
			rss[j] = (uint32_t)rw(p->seed, g, 3);
		if (p->pkt_len)
			p->pkt_len[j] = len;
	}
	return 0;
}
