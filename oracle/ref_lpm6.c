/*
 * ref_lpm6.c -- emits the reference's own IPv6 LPM known-answer data:
 * the 1000-rule large_route_table of test/testcne/lpm6_data_test.h and the
 * IPs generate_large_ips_table() derives from it, each with the next hop the
 * reference's brute-force get_next_hop() (lpm6_data_test.h:1100-1123)
 * assigns.  Compiled from the reference header in place (oracle/Makefile,
 * output in oracle/_ref/); used only by tools/gen_golden.py.  TEST ONLY.
 * Output (stdout, binary): u32 n_rules, n_rules x {16B ip, u8 depth, u8 nh},
 * u32 n_ips, n_ips x {16B ip, u8 nh}.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <cne_common.h>
#include "lpm6_data_test.h"

int main(int argc, char **argv)
{
    long seed = argc > 1 ? atol(argv[1]) : 0x43444E50L;
    srand48(seed);
    generate_large_ips_table(1);
    uint32_t nr = NUM_ROUTE_ENTRIES, ni = NUM_IPS_ENTRIES;
    fwrite(&nr, 4, 1, stdout);
    for (uint32_t i = 0; i < nr; i++) {
        fwrite(large_route_table[i].ip, 16, 1, stdout);
        fwrite(&large_route_table[i].depth, 1, 1, stdout);
        fwrite(&large_route_table[i].next_hop, 1, 1, stdout);
    }
    fwrite(&ni, 4, 1, stdout);
    for (uint32_t i = 0; i < ni; i++) {
        fwrite(large_ips_table[i].ip, 16, 1, stdout);
        fwrite(&large_ips_table[i].next_hop, 1, 1, stdout);
    }
    return 0;
}
