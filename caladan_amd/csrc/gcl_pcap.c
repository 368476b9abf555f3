/*
 * gcl_pcap.c - trace ingest for rx replay: classic libpcap
 * files (LINKTYPE_ETHERNET) to and from the batch layout gcl_classify reads.
 *
 * The reference has no trace reader: its traffic comes from the NIC or from
 * the Rust loadgen.  A loaded trace is one packed host buffer, every frame at
 * a 16-byte-aligned offset (the alignment the classifier's 16-B header loads
 * need, like mbuf data at RTE_PKTMBUF_HEADROOM), with per-packet offsets,
 * captured lengths and timestamps -- ready for gcl_classify_host(ZEROCOPY)
 * once registered with gcl_host_register.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "../../include/gcl_pcap.h"

#define PCAP_MAGIC_US 0xA1B2C3D4u
#define PCAP_MAGIC_NS 0xA1B23C4Du
#define LINKTYPE_ETHERNET 1
/* largest capture loaded: pkt_len is the u16 rte_pktmbuf_pkt_len, and the
 * largest frame the reference handles is ETH_MAX_LEN_JUMBO (inc/net/ethernet.h:18).
 * Longer records (captures on lo, MTU 65536, or of GRO/TSO super-frames with
 * snaplen 262144) are skipped and counted in gcl_trace.skipped, not loaded. */
#define PCAP_MAX_INCL 0xFFFFu

struct pcap_file_hdr {
	uint32_t magic;
	uint16_t vmaj, vmin;
	int32_t thiszone;
	uint32_t sigfigs, snaplen, linktype;
};

struct pcap_rec_hdr {
	uint32_t ts_sec, ts_frac, incl_len, orig_len;
};

static uint32_t bswap32_(uint32_t x) { return __builtin_bswap32(x); }
static uint16_t bswap16_(uint16_t x) { return (uint16_t)(x << 8 | x >> 8); }

int gcl_pcap_write(const char *path, const uint8_t *frames, uint64_t stride,
                   const uint64_t *offs, const uint16_t *pkt_len, const uint64_t *ts_ns,
                   uint64_t n, uint32_t snaplen)
{
	struct pcap_file_hdr fh = {PCAP_MAGIC_NS, 2, 4, 0, 0, snaplen ? snaplen : 65535,
	                           LINKTYPE_ETHERNET};
	FILE *f;

	if (!path || !frames || !pkt_len || (!offs && !stride))
		return -EINVAL;
	f = fopen(path, "wb");
	if (!f)
		return -errno;
	if (fwrite(&fh, sizeof(fh), 1, f) != 1)
		goto io;
	for (uint64_t i = 0; i < n; i++) {
		uint64_t t = ts_ns ? ts_ns[i] : i * 1000;
		uint32_t len = pkt_len[i], incl = len < fh.snaplen ? len : fh.snaplen;
		struct pcap_rec_hdr rh = {(uint32_t)(t / 1000000000ull), (uint32_t)(t % 1000000000ull),
		                          incl, len};
		const uint8_t *p = frames + (offs ? offs[i] : i * stride);
		if (fwrite(&rh, sizeof(rh), 1, f) != 1 || fwrite(p, 1, incl, f) != incl)
			goto io;
	}
	if (fclose(f))
		return -EIO;
	return 0;
io:
	fclose(f);
	return -EIO;
}

static uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) & ~(a - 1); }

int gcl_pcap_load(const char *path, struct gcl_trace *t, uint64_t max_pkts)
{
	struct pcap_file_hdr fh;
	struct pcap_rec_hdr rh;
	struct stat st;
	FILE *f;
	int swap, ns, ret = 0;
	uint64_t n = 0, bytes = 0, cap_pkts, cap_bytes, pos, fsize;

	if (!path || !t)
		return -EINVAL;
	memset(t, 0, sizeof(*t));
	f = fopen(path, "rb");
	if (!f)
		return -errno;
	if (fstat(fileno(f), &st) || !S_ISREG(st.st_mode)) {
		fclose(f);
		return -EINVAL;
	}
	fsize = (uint64_t)st.st_size;
	if (fread(&fh, sizeof(fh), 1, f) != 1) {
		fclose(f);
		return -EPROTO;
	}
	swap = fh.magic == bswap32_(PCAP_MAGIC_US) || fh.magic == bswap32_(PCAP_MAGIC_NS);
	if (swap) {
		fh.magic = bswap32_(fh.magic);
		fh.linktype = bswap32_(fh.linktype);
		fh.vmaj = bswap16_(fh.vmaj);
	}
	if ((fh.magic != PCAP_MAGIC_US && fh.magic != PCAP_MAGIC_NS) || fh.vmaj != 2 ||
	    (fh.linktype & 0xFFFF) != LINKTYPE_ETHERNET) {
		fclose(f);
		return -EPROTO;
	}
	ns = fh.magic == PCAP_MAGIC_NS;
	pos = sizeof(fh);

	/* pass 1: size the packed buffer; every record must lie inside the file
	 * (fseek past EOF succeeds, so the bound is checked against its size) */
	uint64_t skipped = 0;
	while ((!max_pkts || n < max_pkts) && fread(&rh, sizeof(rh), 1, f) == 1) {
		uint32_t incl = swap ? bswap32_(rh.incl_len) : rh.incl_len;
		pos += sizeof(rh);
		if (incl > fsize - pos || fseeko(f, incl, SEEK_CUR)) {
			fclose(f);
			return -EPROTO;
		}
		pos += incl;
		if (incl > PCAP_MAX_INCL) { /* too long for a u16 pkt_len: skipped */
			skipped++;
			continue;
		}
		bytes += align_up(incl ? incl : 1, 16);
		n++;
	}
	if ((!max_pkts || n < max_pkts) && pos != fsize) { /* a cut-off record header */
		fclose(f);
		return -EPROTO;
	}
	cap_pkts = n ? n : 1;
	cap_bytes = bytes + GCL_PCAP_TAIL_PAD;
	if (posix_memalign((void **)&t->frames, 1 << 21, align_up(cap_bytes, 1 << 21)) ||
	    !(t->offs = malloc(cap_pkts * sizeof(uint64_t))) ||
	    !(t->pkt_len = malloc(cap_pkts * sizeof(uint16_t))) ||
	    !(t->orig_len = malloc(cap_pkts * sizeof(uint32_t))) ||
	    !(t->ts_ns = malloc(cap_pkts * sizeof(uint64_t)))) {
		fclose(f);
		gcl_pcap_free(t);
		return -ENOMEM;
	}
	t->alloc_len = align_up(cap_bytes, 1 << 21);
	memset(t->frames, 0, t->alloc_len);

	/* pass 2: copy frames to 16-B-aligned offsets.  The records are re-read,
	 * so each one is bounded again against the buffer pass 1 sized: a file
	 * rewritten in between gives -EPROTO, never a write past the buffer. */
	if (fseeko(f, sizeof(fh), SEEK_SET)) {
		fclose(f);
		gcl_pcap_free(t);
		return -EIO;
	}
	uint64_t off = 0;
	for (uint64_t i = 0; i < n;) {
		if (fread(&rh, sizeof(rh), 1, f) != 1) {
			ret = -EIO;
			break;
		}
		uint32_t incl = swap ? bswap32_(rh.incl_len) : rh.incl_len;
		if (incl > PCAP_MAX_INCL) { /* skipped in pass 1 too */
			if (fseeko(f, incl, SEEK_CUR)) {
				ret = -EIO;
				break;
			}
			continue;
		}
		uint32_t orig = swap ? bswap32_(rh.orig_len) : rh.orig_len;
		uint32_t sec = swap ? bswap32_(rh.ts_sec) : rh.ts_sec;
		uint32_t frac = swap ? bswap32_(rh.ts_frac) : rh.ts_frac;
		uint64_t sz = align_up(incl ? incl : 1, 16);
		if (incl > PCAP_MAX_INCL || sz > bytes - off) {
			ret = -EPROTO;
			break;
		}
		if (incl && fread(t->frames + off, 1, incl, f) != incl) {
			ret = -EIO;
			break;
		}
		t->offs[i] = off;
		t->pkt_len[i] = (uint16_t)incl;
		t->orig_len[i] = orig;
		t->ts_ns[i] = (uint64_t)sec * 1000000000ull + (ns ? frac : (uint64_t)frac * 1000ull);
		off += sz;
		i++;
	}
	fclose(f);
	if (ret) {
		gcl_pcap_free(t);
		return ret;
	}
	t->n = n;
	t->skipped = skipped;
	t->frames_len = off + GCL_PCAP_TAIL_PAD;
	return 0;
}

void gcl_pcap_free(struct gcl_trace *t)
{
	if (!t)
		return;
	free(t->frames);
	free(t->offs);
	free(t->pkt_len);
	free(t->orig_len);
	free(t->ts_ns);
	memset(t, 0, sizeof(*t));
}
