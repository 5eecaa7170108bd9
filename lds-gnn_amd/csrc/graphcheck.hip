// Census of a captured HIP graph's nodes by type, so that the host side can
// refuse a captured step or window that holds anything but kernel launches
// (and the empty nodes a capture inserts at stream joins) before it is ever
// instantiated or replayed.  Round 2 saw a replayed step graph fault on a
// captured hipMemsetAsync node; every memset the engine needs is now a kernel
// (sampler.hip zero_ints_kernel), and this check keeps it that way.
#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/ldsgnn.h"
#include "common.hpp"

extern "C" int lds_graph_node_census(void* graph, int* counts, int ncounts) {
    LDS_CHECK_ARG(graph != nullptr && counts != nullptr && ncounts > 0);
    for (int i = 0; i < ncounts; ++i) counts[i] = 0;
    hipGraph_t g = reinterpret_cast<hipGraph_t>(graph);
    size_t num = 0;
    hipError_t e = hipGraphGetNodes(g, nullptr, &num);
    if (e != hipSuccess) return (int)e;
    std::vector<hipGraphNode_t> nodes(num);
    if (num > 0) {
        e = hipGraphGetNodes(g, nodes.data(), &num);
        if (e != hipSuccess) return (int)e;
    }
    for (size_t i = 0; i < num; ++i) {
        hipGraphNodeType t;
        e = hipGraphNodeGetType(nodes[i], &t);
        if (e != hipSuccess) return (int)e;
        const int ti = (int)t;
        counts[(ti >= 0 && ti < ncounts - 1) ? ti : ncounts - 1] += 1;  // last slot: types past the array
    }
    return 0;
}

extern "C" int lds_graph_upload(void* graph_exec, void* stream) {
    LDS_CHECK_ARG(graph_exec != nullptr);
    return (int)hipGraphUpload(reinterpret_cast<hipGraphExec_t>(graph_exec), (hipStream_t)stream);
}
