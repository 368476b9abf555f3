/*
 * ref_trans.c - test infrastructure (oracle/_ref only, never linked into the
 * product): the reference's own transport demux hashes trans_hash_5tuple /
 * trans_hash_3tuple (/root/reference/runtime/net/transport.c:29-42), compiled
 * where they lie.
 *
 * oracle/Makefile passes the reference file's path as REF_TRANSPORT_C and
 * this file #includes it unmodified, against the reference's own headers.
 * The two functions are static inline and read the file's static
 * trans_seed (a runtime sets it at start-up, transport.c:26); this file sets
 * it per call and exports one entry point.  The rest of transport.c is
 * unreachable and dropped by --gc-sections; the library links with
 * --no-undefined, so nothing is stubbed.
 */
#include REF_TRANSPORT_C

/* trans_hash_5tuple(proto, laddr, raddr) and trans_hash_3tuple(proto, laddr)
 * with trans_seed = @seed; addresses and ports in host order */
__attribute__((visibility("default"))) void ref_trans_hash(uint32_t seed, uint8_t proto,
                                                           uint32_t lip, uint16_t lport,
                                                           uint32_t rip, uint16_t rport,
                                                           uint32_t out[2])
{
	struct netaddr l = {.ip = lip, .port = lport}, r = {.ip = rip, .port = rport};

	trans_seed = seed;
	out[0] = trans_hash_5tuple(proto, l, r);
	out[1] = trans_hash_3tuple(proto, l);
}
