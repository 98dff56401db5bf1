#pragma once
// lab forwarding header: the product 128-class IPM kernel (renamed per variant by ipm_variant.hip)
#include "k_ipm128x.hpp"
