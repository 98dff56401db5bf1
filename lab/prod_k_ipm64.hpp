#pragma once
// lab forwarding header: the product 64-class IPM kernel (renamed per variant by ipm_variant.hip)
#include "k_ipm64.hpp"
