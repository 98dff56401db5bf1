#pragma once
#include "ipm_v5.hpp"
