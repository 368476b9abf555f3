/*
 * gcl_pcap.h - libpcap trace files <-> rx batches (trace replay).
 */
#ifndef GCL_PCAP_H
#define GCL_PCAP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* zeroed bytes after the last frame, so every frame has a full 64-B granule */
#define GCL_PCAP_TAIL_PAD 128

/* A trace loaded into one packed host buffer. */
struct gcl_trace {
	uint8_t  *frames;     /* 2 MiB-aligned; frame i at frames + offs[i] (16-B aligned) */
	uint64_t  frames_len; /* bytes holding frames (+ GCL_PCAP_TAIL_PAD zero bytes) */
	uint64_t  alloc_len;  /* bytes allocated at frames (for gcl_host_register) */
	uint64_t *offs;       /* u64[n] */
	uint16_t *pkt_len;    /* u16[n] captured length (rte_pktmbuf_pkt_len) */
	uint32_t *orig_len;   /* u32[n] length on the wire */
	uint64_t *ts_ns;      /* u64[n] capture time */
	uint64_t  n;
	uint64_t  skipped;    /* records not loaded: captures longer than 65535 bytes */
};

/*
 * gcl_pcap_load - read a classic pcap file (either byte order, micro- or
 * nanosecond timestamps, LINKTYPE_ETHERNET) into @t; at most @max_pkts
 * packets (0 = all).  A record whose capture is longer than 65535 bytes
 * (pkt_len is a u16, and the largest frame the reference handles is
 * ETH_MAX_LEN_JUMBO; such records come from captures on lo or of GRO/TSO
 * super-frames) is skipped and counted in @t->skipped.  Returns 0, -EPROTO
 * (not an Ethernet pcap, a record running past the end of the file, or a
 * cut-off record header), -EINVAL (not a regular file), -ENOMEM, -EIO or
 * -errno from fopen.
 */
int gcl_pcap_load(const char *path, struct gcl_trace *t, uint64_t max_pkts);
void gcl_pcap_free(struct gcl_trace *t);

/*
 * gcl_pcap_write - write @n frames as a nanosecond pcap: frame i is at
 * frames + offs[i] (or i * stride when @offs is NULL) and is @pkt_len[i]
 * bytes long; @ts_ns may be NULL (1 us apart).  Captures are cut at @snaplen
 * (0 = 65535).
 */
int gcl_pcap_write(const char *path, const uint8_t *frames, uint64_t stride,
                   const uint64_t *offs, const uint16_t *pkt_len, const uint64_t *ts_ns,
                   uint64_t n, uint32_t snaplen);

#ifdef __cplusplus
}
#endif

#endif
