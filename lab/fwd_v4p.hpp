#pragma once
#include "ipm_v4prod.hpp"
