// Launch-configuration inputs of the executor (host only).
//
// Reference: MADRONA_MWGPU_EXEC_CONFIG_OVERRIDE = "threads,blocksPerSM,numSMs"
// (processExecConfigOverride, src/mw/cuda_exec.cpp:1401-1438) picks the
// default megakernel configuration, and MADRONA_MWGPU_EXEC_CONFIG_FILE names a
// JSON object {"<node index>": <blocks per SM>, ...} (processExecConfigFile,
// :1460-1517) that picks one per taskgraph node; malformed input is FATAL.
//
// Here every node is its own set of kernels with compile-time block sizes, so
// the configuration that remains per node is the grid: blocks per CU for the
// node's grid-stride and persistent kernels (LaunchCtx::capGrid /
// persistentGrid), and the CU count grids are sized for.  The thread count of
// the override is accepted for format compatibility and otherwise unused.
#include <madrona/launch_config.hpp>

#include <cctype>
#include <charconv>
#include <climits>
#include <cstring>
#include <stdexcept>

namespace madrona {

static bool parseU32(const char *b, const char *e, uint32_t &out)
{
    while (b < e && std::isspace((unsigned char)*b)) b++;
    while (e > b && std::isspace((unsigned char)e[-1])) e--;
    if (b == e) return false;
    auto r = std::from_chars(b, e, out);
    return r.ec == std::errc {} && r.ptr == e;
}

ExecConfigOverride parseExecConfigOverride(const char *s)
{
    auto err = []() -> ExecConfigOverride {
        throw std::runtime_error("MADRONA_MWGPU_EXEC_CONFIG_OVERRIDE format invalid "
                                 "(expected \"threads,blocksPerCU,numCUs\")");
    };
    const char *c1 = std::strchr(s, ',');
    if (!c1) return err();
    const char *c2 = std::strchr(c1 + 1, ',');
    if (!c2) return err();
    ExecConfigOverride o {};
    if (!parseU32(s, c1, o.numThreads) || !parseU32(c1 + 1, c2, o.blocksPerCU) ||
        !parseU32(c2 + 1, s + std::strlen(s), o.numCUs)) {
        return err();
    }
    if (o.blocksPerCU > (uint32_t)kMaxBlocksPerCU || o.numCUs > (uint32_t)kMaxLaunchCUs) {
        throw std::runtime_error("MADRONA_MWGPU_EXEC_CONFIG_OVERRIDE out of range "
                                 "(blocksPerCU <= 64, numCUs <= 65536)");
    }
    return o;
}

// A flat JSON object with string keys holding node indices and unsigned
// integer values; whitespace anywhere between tokens.
std::vector<NodeBlocks> parseExecConfigFile(const std::string &text)
{
    auto err = [](const char *what) {
        throw std::runtime_error(std::string("MADRONA_MWGPU_EXEC_CONFIG_FILE points to invalid file: ") +
                                 what);
    };
    std::vector<NodeBlocks> out;
    size_t i = 0;
    const size_t n = text.size();
    auto skip = [&]() {
        while (i < n && std::isspace((unsigned char)text[i])) i++;
    };
    skip();
    if (i >= n || text[i] != '{') err("expected '{'");
    i++;
    skip();
    if (i < n && text[i] == '}') {
        i++;
    } else {
        for (;;) {
            skip();
            if (i >= n || text[i] != '"') err("expected a quoted node index");
            const size_t kb = ++i;
            while (i < n && text[i] != '"') i++;
            if (i >= n) err("unterminated key");
            uint32_t node = 0;
            if (!parseU32(text.data() + kb, text.data() + i, node)) err("key is not a node index");
            if (node > (uint32_t)INT32_MAX) err("node index out of range");
            i++;
            skip();
            if (i >= n || text[i] != ':') err("expected ':'");
            i++;
            skip();
            const size_t vb = i;
            while (i < n && std::isdigit((unsigned char)text[i])) i++;
            uint32_t blocks = 0;
            if (!parseU32(text.data() + vb, text.data() + i, blocks)) err("value is not a block count");
            if (blocks > (uint32_t)kMaxBlocksPerCU) err("block count out of range (at most 64 per CU)");
            out.push_back(NodeBlocks { (int32_t)node, (int32_t)blocks });
            skip();
            if (i < n && text[i] == ',') {
                i++;
                continue;
            }
            if (i < n && text[i] == '}') {
                i++;
                break;
            }
            err("expected ',' or '}'");
        }
    }
    skip();
    if (i != n) err("trailing characters");
    return out;
}

}
