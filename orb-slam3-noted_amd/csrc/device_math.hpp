// device_math.hpp — HIP include wrapper of device_math_core.hpp (bit-exact device
// restatements of glibc sincosf, cv::fastAtan2 and cvRound).
#pragma once

#include <hip/hip_runtime.h>

#include "device_math_core.hpp"
