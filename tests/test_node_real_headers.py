"""The GPU graph node sources (cndp_amd/node/*.c) compiled against CNDP's own
graph, pktmbuf, pktdev and cnet headers (lib/usr/clib/graph/cne_graph.h,
cne_graph_worker.h:50-80 -- the real struct cne_node with its cache-aligned
ctx[CNE_NODE_CTX_SZ] -- and :460-540's stream ops), not the test harness's
stand-ins: every type, field and call the nodes use must exist there with a
compatible signature, and each node's context must fit ctx
(_Static_assert in the sources).  A compile check only (-fsyntax-only): the
reference's meson-generated cne_build_config.h and libbsd's headers are absent
here, so the test supplies the few definitions they would (the version macros,
strlcpy / strlcat prototypes, sys/queue.h; -D_GNU_SOURCE as meson.build:333-334) in a
temporary directory.  Runs where the
reference tree is present (this container), skipped elsewhere."""
import glob
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = "/root/reference"
NODES = ["ip4_lookup_gpu.c", "ip4_rewrite_gpu.c", "pktdev_rx_gpu.c", "eth_rx_gpu.c"]


@pytest.fixture(scope="module")
def ref_includes(tmp_path_factory):
    if not os.path.isdir(os.path.join(REF, "lib", "usr", "clib", "graph")):
        pytest.skip("reference tree absent")
    d = tmp_path_factory.mktemp("forced")
    (d / "cne_build_config.h").write_text(
        "#pragma once\n#define CNE_VER_PREFIX \"CNDP\"\n#define CNE_VER_SUFFIX \"\"\n#define CNE_VER_YEAR 25\n"
        "#define CNE_VER_MONTH 8\n#define CNE_VER_MINOR 0\n#define CNE_VER_RELEASE 0\n")
    (d / "bsd" / "sys").mkdir(parents=True)
    (d / "bsd" / "string.h").write_text(
        "#pragma once\n#include <string.h>\nsize_t strlcpy(char *dst, const char *src, size_t size);\n"
        "size_t strlcat(char *dst, const char *src, size_t size);\n")
    (d / "bsd" / "sys" / "queue.h").write_text("#pragma once\n#include <sys/queue.h>\n")
    dirs = sorted({os.path.dirname(h) for h in glob.glob(os.path.join(REF, "lib", "**", "*.h"), recursive=True)})
    return ["-I" + str(d)] + ["-I" + x for x in dirs]


@pytest.mark.parametrize("src", NODES)
def test_node_compiles_against_cndp_headers(ref_includes, src):
    # the real cne_graph_worker.h / pktdev_rx_priv.h / eth_rx_priv.h are found
    # through the reference include paths: none of tests/node_harness is used
    cmd = ["gcc", "-fsyntax-only", "-std=gnu11", "-D_GNU_SOURCE", "-Wall", "-Werror=implicit-function-declaration",
           "-Werror=incompatible-pointer-types", "-Werror=int-conversion", *ref_includes,
           "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "cndp_amd", "node", src)]
    p = subprocess.run(cmd, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "node_harness" not in p.stderr
    # the reference's worker header defines the node context the sources assert against
    assert "CNE_NODE_CTX_SZ" in open(os.path.join(REF, "lib", "usr", "clib", "graph", "cne_graph_worker.h")).read()
