// Caller.h — the reference's driver API (BlockMatching/Caller.h:8-10), kept for drop-in callers.
// Only singleFrame() is on the matching path; remapTest()/cvtColorTest() are the reference's
// rectification/gray demos (out of scope) and print a notice here.
#pragma once
void singleFrame();
void remapTest();
void cvtColorTest();
