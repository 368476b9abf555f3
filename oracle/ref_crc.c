/*
 * ref_crc.c - exports the reference's own CRC32C hash helpers, which are
 * header-only inline functions (inc/base/hash.h:23-40 over crc32q,
 * inc/asm/ops.h:77-80), so the oracle's restatement can be checked against
 * them.  Compiled only when /root/reference is mounted (oracle/Makefile).
 */
#include <stdint.h>

#include <base/hash.h>

uint32_t ref_crc32c_one(uint32_t seed, uint64_t val)
{
	return hash_crc32c_one(seed, val);
}

uint32_t ref_crc32c_two(uint32_t seed, uint64_t a, uint64_t b)
{
	return hash_crc32c_two(seed, a, b);
}
