// base::registerTypes (reference src/core/base.cpp:7-17).
#include <madrona/components.hpp>
#include <madrona/state.hpp>

namespace madrona::base {

void registerTypes(ECSRegistry &registry)
{
    registry.registerComponent<Position>();
    registry.registerComponent<Rotation>();
    registry.registerComponent<Scale>();
    registry.registerComponent<ObjectID>();
}

}
