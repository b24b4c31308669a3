// Caller.h — the reference's driver API (BlockMatching/Caller.h:8-10), kept for drop-in callers.
#pragma once
void singleFrame();
void remapTest();
void cvtColorTest();
void blockMatchingApiTest();   // not in the reference's Caller.h: BlockMatching.h through the adapter
