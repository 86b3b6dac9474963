#!/usr/bin/env python3
"""Write tests/golden/ptype_ref.json from the REFERENCE's own source text
(run where /root/reference exists):

  * every CNE_PTYPE_* value (lib/core/pktmbuf/pktmbuf_ptype.h),
  * the ptype node's edge ids (enum ptype_next_nodes, lib/cnet/ptype/ptype_priv.h,
    with CNET_ENABLE_IP6 = 1 as cnet builds it),
  * its next-node table p_nxt[_PTYPE_MASK + 1] (lib/cnet/ptype/ptype.c:20-46):
    the designated initializers evaluated over those constants,
  * cne_get_ptype's lookup tables (lib/core/pktmbuf/pktmbuf_ptype.c:279-321,
    :372-380): IPv4 version/IHL byte -> L3 type, IPv6 next header -> the
    IPv6 / IPv6-with-extensions offset, protocol -> L4 type, GRE flags ->
    option length.  IPPROTO_* are the C library's (netinet/in.h) numbers,
  * what eth_rx's mbuf_update writes them into (lib/cnet/eth/eth_rx.c:35-63):
    the tx_offload bit-field layout (the CNE_MBUF_*_BITS / _OFS enum of
    lib/core/pktmbuf/pktmbuf_offload.h) and the CNE_MBUF_TYPE_* ol_flags bits,
  * the cnet input nodes' edge ids (ip4_input_priv.h / ip6_input_priv.h), the
    next-index shift of a cnet FIB value (cnet_route4.h / cnet_route6.h) and the
    cnet node names (lib/cnet/incs/cnet_node_names.h).

pktmbuf_ptype.c / ptype.c cannot be compiled here (pktmbuf.h needs
<bsd/string.h>), so the table is taken from the text the compiler would
read: the macros and initializers are evaluated, nothing is restated.  The
fixture is data: names, numbers, and the non-zero table entries.

    python tools/gen_ptype_golden.py
"""
from __future__ import annotations

import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("CNDP_REF", "/root/reference")
OUT = os.path.join(ROOT, "tests", "golden", "ptype_ref.json")


def strip_if(text: str, macro: str, value: bool) -> str:
    """Keep or drop `#if MACRO ... #endif` blocks (no #else in these files)."""
    out, keep = [], [True]
    for line in text.split("\n"):
        s = line.strip()
        if s.startswith("#if"):
            keep.append(keep[-1] and (value if macro in s else True))
            continue
        if s.startswith("#endif"):
            keep.pop()
            continue
        if keep[-1]:
            out.append(line)
    return "\n".join(out)


def main():
    hdr = open(os.path.join(REF, "lib/core/pktmbuf/pktmbuf_ptype.h")).read()
    consts = {m.group(1): int(m.group(2), 16)
              for m in re.finditer(r"#define\s+(CNE_PTYPE_\w+)\s+(0x[0-9a-fA-F]+)", hdr)}
    priv = strip_if(open(os.path.join(REF, "lib/cnet/ptype/ptype_priv.h")).read(), "CNET_ENABLE_IP6", True)
    body = re.search(r"enum\s+ptype_next_nodes\s*\{(.*?)\}", priv, re.S).group(1)
    names = [n.strip() for n in body.replace("\n", " ").split(",") if n.strip()]
    edges = {n: i for i, n in enumerate(names)}
    src = strip_if(open(os.path.join(REF, "lib/cnet/ptype/ptype.c")).read(), "CNET_ENABLE_IP6", True)
    src = src.replace("\\\n", " ")
    macros = {m.group(1): m.group(2) for m in re.finditer(r"#define\s+(_\w+)\s+\((.*?)\)\s*\n", src)}
    env = dict(consts)
    env.update(edges)

    def ev(expr: str) -> int:
        for _ in range(4):  # nested macros
            expr = re.sub(r"\b(_\w+)\b", lambda m: "(" + macros[m.group(1)] + ")" if m.group(1) in macros
                          else m.group(1), expr)
        assert re.fullmatch(r"[\w\s|()]+", expr), expr
        return int(eval(expr, {"__builtins__": {}}, env))

    mask = ev("_PTYPE_MASK")
    init = re.search(r"p_nxt\[_PTYPE_MASK \+ 1\][^=]*=\s*\{(.*?)\};", src, re.S).group(1)
    table = {}
    for m in re.finditer(r"\[([^\]]+)\]\s*=\s*(\w+)", init):
        table[ev(m.group(1))] = edges[m.group(2)]
    # cne_get_ptype's static tables, by array name (the first, outer, ones)
    ptc = open(os.path.join(REF, "lib/core/pktmbuf/pktmbuf_ptype.c")).read()
    ipproto = {"IPPROTO_HOPOPTS": 0, "IPPROTO_TCP": 6, "IPPROTO_UDP": 17, "IPPROTO_ROUTING": 43,
               "IPPROTO_FRAGMENT": 44, "IPPROTO_ESP": 50, "IPPROTO_AH": 51, "IPPROTO_DSTOPTS": 60,
               "IPPROTO_SCTP": 132}
    env.update(ipproto)

    def arr(name: str) -> dict:
        body = re.search(re.escape(name) + r"\[\d+\]\s*=\s*\{(.*?)\};", ptc, re.S).group(1)
        out = {}
        for m in re.finditer(r"\[([^\]]+)\]\s*=\s*([^,\n]+)", body):
            k = m.group(1).strip()
            key = int(k, 16) if k.startswith("0x") else ev(k)
            v = m.group(2).strip()
            assert re.fullmatch(r"[\w\s|()+-]+", v), v
            out[key] = int(eval(v, {"__builtins__": {}}, env))
        return out

    tables = {"l3_ip_by_ihl": arr("ptype_l3_ip_proto_map"), "l4_by_proto": arr("ptype_l4_proto"),
              "ip6_ext_by_proto": arr("ip6_ext_proto_map"), "gre_opt_len": arr("opt_len")}
    off = open(os.path.join(REF, "lib/core/pktmbuf/pktmbuf_offload.h")).read()
    oenum = re.search(r"enum\s*\{([^}]*CNE_MBUF_L2_LEN_BITS[^}]*)\}", off, re.S).group(1)
    layout = {}
    for m in re.finditer(r"(CNE_MBUF_\w+)\s*=\s*([^,]+),", oenum):
        if "sizeof" in m.group(2):
            continue
        expr = m.group(2)
        for k, v in layout.items():
            expr = re.sub(r"\b" + k + r"\b", str(v), expr)
        assert re.fullmatch(r"[\d\s+()-]+", expr), expr
        layout[m.group(1)] = int(eval(expr, {"__builtins__": {}}, {}))
    olf = {m.group(1): 1 << int(m.group(2))
           for m in re.finditer(r"#define\s+(CNE_MBUF_TYPE_\w+)\s+\(1ULL << (\d+)\)", off)}
    inp = {}
    for f, en in (("lib/cnet/ipv4/ip4_input_priv.h", "cne_node_ip4_input_next"),
                  ("lib/cnet/ipv6/ip6_input_priv.h", "cne_node_ip6_input_next")):
        t = open(os.path.join(REF, f)).read()
        body = re.search(r"enum\s+" + en + r"\s*\{(.*?)\}", t, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        for i, nm in enumerate(x.strip() for x in body.split(",") if x.strip()):
            inp[nm] = i
    shift = {}
    for f, nm in (("lib/cnet/route/cnet_route4.h", "RT4_NEXT_INDEX_SHIFT"),
                  ("lib/cnet/route/cnet_route6.h", "RT6_NEXT_INDEX_SHIFT")):
        shift[nm] = int(re.search(r"#define\s+" + nm + r"\s+(\d+)", open(os.path.join(REF, f)).read()).group(1))
    names = dict(re.findall(r'#define\s+(\w+_NODE_NAME)\s+"([^"]+)"',
                            open(os.path.join(REF, "lib/cnet/incs/cnet_node_names.h")).read()))
    res = {"source": "lib/core/pktmbuf/pktmbuf_ptype.h, lib/cnet/ptype/ptype_priv.h (CNET_ENABLE_IP6=1), "
                     "lib/cnet/ptype/ptype.c:20-46, lib/core/pktmbuf/pktmbuf_ptype.c:279-321,372-380, "
                     "lib/core/pktmbuf/pktmbuf_offload.h:365-412, "
                     "lib/cnet/ipv{4,6}/ip{4,6}_input_priv.h, lib/cnet/route/cnet_route{4,6}.h:28, "
                     "lib/cnet/incs/cnet_node_names.h (CNDP v25.08.0)",
           "ptype_consts": consts, "ptype_next": edges, "pnxt_mask": mask,
           "pnxt": {f"{k:#06x}": v for k, v in sorted(table.items())},
           "get_ptype_tables": {n: {str(k): v for k, v in sorted(t.items())} for n, t in tables.items()},
           "tx_offload_layout": layout, "ol_flags_type": olf,
           "input_next": inp, "next_index_shift": shift, "cnet_node_names": names}
    with open(OUT, "w") as f:
        json.dump(res, f, indent=1)
    print(f"wrote {OUT}: {len(consts)} constants, {len(edges)} edges, {len(table)} table entries, mask {mask:#x}")


if __name__ == "__main__":
    main()
