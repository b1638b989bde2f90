// tl/tl.h — umbrella header included by every generated gfx950 kernel.
#pragma once
#include "common.h"
#include "copy.h"
#include "gemm.h"
#include "gemm_quad.h"
#include "reduce.h"
#include "atomic.h"
#include "swizzle.h"
#include "debug.h"
#include "mesh.h"
#include "ep.h"
#include "gemv.h"
