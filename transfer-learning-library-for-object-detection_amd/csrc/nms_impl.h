// Internal NMS launcher shared by the NMS entry point and the proposal pipeline.
#pragma once
#include "common.h"

namespace tlod {
size_t nms_ws_bytes(int n);
int nms_launch(const float* boxes, int n, int dim, float thresh, int max_keep, int32_t* keep,
               int32_t* num_keep, void* ws, size_t ws_bytes, hipStream_t s);
}  // namespace tlod
