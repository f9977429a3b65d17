// Per-node launch configuration inputs (see csrc/runtime/launch_config.cpp;
// reference src/mw/cuda_exec.cpp:1401-1560).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace madrona {

// Bounds of every blocks-per-CU value (parsers, setNodeBlocksPerCU) and of
// the CU count a grid is sized for: grids stay far below 2^31 blocks.
inline constexpr int32_t kMaxBlocksPerCU = 64;
inline constexpr int32_t kMaxLaunchCUs = 65536;

struct ExecConfigOverride {
    uint32_t numThreads;     // accepted for format compatibility
    uint32_t blocksPerCU;    // default blocks per CU of every node
    uint32_t numCUs;         // CUs grids are sized for (0 = the device's)
};

struct NodeBlocks {
    int32_t node;
    int32_t blocksPerCU;
};

// Both throw std::runtime_error on malformed input (the reference FATALs).
ExecConfigOverride parseExecConfigOverride(const char *s);
std::vector<NodeBlocks> parseExecConfigFile(const std::string &text);

}
