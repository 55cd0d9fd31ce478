// Host compilation of device_math.hpp (for the oracle's self-checks) without HIP headers.
#pragma once
#include <cmath>
#include <cstdint>
#define __host__
#define __device__
#include "device_math_core.hpp"
#undef __host__
#undef __device__
