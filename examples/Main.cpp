// Main.cpp — the reference's entry point (BlockMatching/Main.cpp:3-9), unchanged in shape.
// SM_DEMO selects which Caller.h demo runs: singleFrame (default), remapTest or cvtColorTest.
#include <cstdlib>
#include <cstring>
#include "Caller.h"

int main() {
    const char* demo = std::getenv("SM_DEMO");
    if (demo && std::strcmp(demo, "remapTest") == 0) {
        remapTest();
    } else if (demo && std::strcmp(demo, "cvtColorTest") == 0) {
        cvtColorTest();
    } else if (demo && std::strcmp(demo, "blockMatchingApiTest") == 0) {
        blockMatchingApiTest();
    } else {
        singleFrame();
    }
    return 0;
}
