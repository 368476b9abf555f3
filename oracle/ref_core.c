/*
 * ref_core.c - test infrastructure (oracle/_ref only, never linked into the
 * product): the reference's own do_toeplitz
 * (/root/reference/runtime/net/core.c:120-139) and ip_hdr_supported
 * (core.c:203-209, which frames reach the transport demux), compiled where
 * they lie.
 *
 * oracle/Makefile passes the reference file's path as REF_CORE_C and this
 * file #includes it unmodified, against the reference's own headers
 * (inc/, runtime/, runtime/net/).  do_toeplitz is static and reads the RSS
 * key from the runtime's `iok` global (runtime/defs.h:193-199), which the
 * runtime fills from the iokernel's shared memory at start-up; this file
 * defines that global -- the function's input, as tests/ set it -- and
 * exports entry points for the two static functions.  Nothing the reference references is stubbed:
 * the rest of core.c is unreachable from the export and dropped by
 * --gc-sections, and the library links with --no-undefined.
 */
#include REF_CORE_C

struct iokernel_control iok;
static struct iokernel_info ref_info;

/* do_toeplitz(saddr, daddr, sport, dport) (host-order fields) with RSS key
 * @key (@key_len <= 52 bytes, iokernel_info.rss_key) */
__attribute__((visibility("default"))) uint32_t ref_do_toeplitz(const uint8_t *key,
                                                                uint32_t key_len,
                                                                uint32_t saddr, uint32_t daddr,
                                                                uint16_t sport, uint16_t dport)
{
	memset(ref_info.rss_key, 0, sizeof(ref_info.rss_key));
	memcpy(ref_info.rss_key, key,
	       key_len < sizeof(ref_info.rss_key) ? key_len : sizeof(ref_info.rss_key));
	ref_info.rss_key_len = key_len;
	iok.iok_info = &ref_info;
	return do_toeplitz(saddr, daddr, sport, dport);
}

/* ip_hdr_supported on the 20-byte IPv4 header at @hdr (wire order) */
__attribute__((visibility("default"))) int ref_ip_hdr_supported(const uint8_t *hdr)
{
	struct ip_hdr ip;

	memcpy(&ip, hdr, sizeof(ip));
	return ip_hdr_supported(&ip);
}
