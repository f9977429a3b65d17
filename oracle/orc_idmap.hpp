// ORACLE (test infrastructure only) — single-threaded restatement of the
// reference generation-checked entity ID allocator,
// include/madrona/impl/id_map_impl.inl:17-332 (ids_per_cache_ = 64,
// include/madrona/impl/id_map.hpp:134).  Lock-free CAS loops collapse to plain
// stores because the oracle is serial; the resulting ID / generation sequence
// is the one a serial caller of the reference observes.
#pragma once

#include <cstdint>
#include <vector>

namespace orc {

struct Entity {
    uint32_t gen;
    int32_t id;
};

struct Loc {
    uint32_t archetype;
    int32_t row;
};

class IDMap {
public:
    static constexpr int32_t idsPerCache = 64;
    static constexpr int32_t sentinel = -1;

    struct Cache {
        int32_t freeHead = sentinel;
        int32_t numFree = 0;
        int32_t overflowHead = sentinel;
        int32_t numOverflow = 0;
    };

    struct Node {
        Loc val;          // overlaps FreeNode {subNext, globalNext}
        uint32_t gen;
        int32_t &subNext() { return *(int32_t *)&val.archetype; }
        int32_t &globalNext() { return val.row; }
    };

    Entity acquireID(Cache &cache)                          // id_map_impl.inl:69-182
    {
        auto assignCached = [this](int32_t *head) {
            int32_t new_id = *head;
            Node &node = nodes_[new_id];
            int32_t num_contiguous = node.globalNext();
            if (num_contiguous == 1) {
                *head = node.subNext();
            } else {
                int32_t next_free = new_id + 1;
                Node &next_node = nodes_[next_free];
                next_node.subNext() = node.subNext();
                next_node.globalNext() = num_contiguous - 1;
                next_node.gen = 0;
                *head = next_free;
            }
            return Entity { node.gen, new_id };
        };

        if (cache.numOverflow > 0) {
            cache.numOverflow -= 1;
            return assignCached(&cache.overflowHead);
        }
        if (cache.numFree > 0) {
            cache.numFree -= 1;
            return assignCached(&cache.freeHead);
        }

        if (globalHead_ != sentinel) {
            int32_t free_ids = globalHead_;
            Node &head_node = nodes_[free_ids];
            globalHead_ = head_node.globalNext();
            head_node.globalNext() = 1;
            cache.freeHead = free_ids;
            cache.numFree = idsPerCache - 1;
            return assignCached(&cache.freeHead);
        }

        int32_t block_start = (int32_t)nodes_.size();
        nodes_.resize(nodes_.size() + idsPerCache);
        Node &assigned = nodes_[block_start];
        assigned.gen = 0;
        Node &next_free = nodes_[block_start + 1];
        next_free.subNext() = sentinel;
        next_free.globalNext() = idsPerCache - 1;
        next_free.gen = 0;
        cache.freeHead = block_start + 1;
        cache.numFree = idsPerCache - 1;
        return Entity { 0, block_start };
    }

    void releaseID(Cache &cache, int32_t id)                // id_map_impl.inl:184-226
    {
        Node &rel = nodes_[id];
        rel.gen += 1;
        rel.globalNext() = 1;

        if (cache.numFree < idsPerCache) {
            rel.subNext() = cache.freeHead;
            cache.freeHead = id;
            cache.numFree += 1;
            return;
        }
        if (cache.numOverflow < idsPerCache) {
            rel.subNext() = cache.overflowHead;
            cache.overflowHead = id;
            cache.numOverflow += 1;
        }
        if (cache.numOverflow == idsPerCache) {
            Node &new_node = nodes_[cache.overflowHead];
            new_node.globalNext() = globalHead_;
            globalHead_ = cache.overflowHead;
            cache.overflowHead = sentinel;
            cache.numOverflow = 0;
        }
    }

    void bulkRelease(Cache &cache, const Entity *keys, int32_t num_keys)  // :228-332
    {
        if (num_keys <= 0) return;
        auto linkToNext = [&](int32_t idx) {
            Node &node = nodes_[keys[idx].id];
            node.gen += 1;
            node.subNext() = keys[idx + 1].id;
            node.globalNext() = 1;
        };

        int32_t base_idx;
        int32_t num_remaining = 0;
        Node *global_tail = nullptr;
        for (base_idx = 0; base_idx < num_keys; base_idx += idsPerCache) {
            num_remaining = num_keys - base_idx;
            if (num_remaining < idsPerCache) break;
            int32_t head_id = keys[base_idx].id;
            for (int32_t sub = 0; sub < idsPerCache; sub++) {
                linkToNext(base_idx + sub);
            }
            Node &last = nodes_[keys[base_idx + idsPerCache - 1].id];
            last.gen += 1;
            last.subNext() = sentinel;
            last.globalNext() = 1;
            if (global_tail) global_tail->globalNext() = head_id;
            global_tail = &nodes_[head_id];
        }

        if (num_remaining != idsPerCache) {
            int32_t start_id = keys[base_idx].id;
            for (int32_t idx = base_idx; idx < num_keys - 1; idx++) linkToNext(idx);
            Node &tail = nodes_[keys[num_keys - 1].id];
            tail.gen += 1;
            tail.globalNext() = 1;
            tail.subNext() = cache.overflowHead;

            int32_t num_from_overflow = idsPerCache - num_remaining;
            if (cache.numOverflow < num_from_overflow) {
                cache.overflowHead = start_id;
                cache.numOverflow += num_remaining;
            } else {
                int32_t next_id = cache.overflowHead;
                Node *overflow_node = nullptr;
                for (int32_t i = 0; i < num_from_overflow; i++) {
                    overflow_node = &nodes_[next_id];
                    next_id = overflow_node->subNext();
                }
                overflow_node->subNext() = sentinel;
                cache.overflowHead = next_id;
                cache.numOverflow -= num_from_overflow;
                if (global_tail) global_tail->globalNext() = start_id;
                global_tail = &nodes_[start_id];
            }
        }

        if (!global_tail) return;
        global_tail->globalNext() = globalHead_;
        globalHead_ = keys[0].id;
    }

    Loc lookup(Entity e) const
    {
        const Node &n = nodes_[e.id];
        if (n.gen != e.gen) return Loc { 0xFFFFFFFFu, 0 };
        return n.val;
    }
    Loc &ref(int32_t id) { return nodes_[id].val; }

private:
    std::vector<Node> nodes_;
    int32_t globalHead_ = sentinel;
};

}
