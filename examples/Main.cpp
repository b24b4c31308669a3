// Main.cpp — the reference's entry point (BlockMatching/Main.cpp:3-9), unchanged in shape.
#include <cstdlib>
#include "Caller.h"

int main() {
    singleFrame();
    if (std::getenv("SM_ALL_DEMOS")) {
        remapTest();
        cvtColorTest();
    }
    return 0;
}
