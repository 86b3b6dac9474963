/*
 * ref_harness.c -- thin driver around the REFERENCE's own header-only code,
 * compiled straight from /root/reference by oracle/Makefile into
 * oracle/_ref/libcndp_ref.so (never committed; it travels to the GPU box as
 * a built artefact).  TEST INFRASTRUCTURE ONLY.
 *
 * Buildable here with gcc and -I paths into the reference tree, no stand-ins:
 *   lib/core/hash/cne_thash.h    cne_softrss / cne_softrss_be /
 *                                cne_convert_rss_key            (:113-191)
 *   lib/include/net/cne_ip.h     cne_ipv4_cksum                 (:131-214)
 * NOT buildable without stand-ins (DESIGN.md §3 records why): dir24_8.h and
 * trie.h (via cne_fib.h -> cne_inet4.h -> <bsd/string.h>, libbsd absent),
 * dir24_8.c / trie.c / cne_rib*.c / cne_fib*.c (generated cne_build_config.h),
 * pktmbuf_ptype.c (libbsd), the graph nodes and cnet.  Their behaviour is
 * restated in oracle.c and pinned by the reference's own test ladders.
 */
#include <stdint.h>

#include <cne_thash.h>
#include <net/cne_ip.h>

uint32_t ref_softrss(uint32_t *tuple, uint32_t len, const uint8_t *key)
{
    return cne_softrss(tuple, len, key);
}

uint32_t ref_softrss_be(uint32_t *tuple, uint32_t len, const uint8_t *key)
{
    return cne_softrss_be(tuple, len, key);
}

void ref_convert_rss_key(const uint8_t *orig, uint8_t *targ, int len)
{
    cne_convert_rss_key((const uint32_t *)(const void *)orig, (uint32_t *)(void *)targ, len);
}

uint16_t ref_ipv4_cksum(const uint8_t *hdr)
{
    return cne_ipv4_cksum((const struct cne_ipv4_hdr *)(const void *)hdr);
}

/* cne_thash_load_v6_addrs (cne_thash.h:130-137) over a raw IPv6 header,
 * returning the 8 host-order address dwords it produces. */
void ref_thash_load_v6(const uint8_t *ip6_hdr, uint32_t out[8])
{
    union cne_thash_tuple t;
    cne_thash_load_v6_addrs((const struct cne_ipv6_hdr *)(const void *)ip6_hdr, &t);
    for (int k = 0; k < 8; k++)
        out[k] = ((const uint32_t *)(const void *)t.v6.src_addr)[k];
}
