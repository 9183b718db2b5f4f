/*
 * liquid.h -- drop-in include name: programs built against liquid-dsp with
 * `-I<liquid>/include` and `#include "liquid.h"` that use only the streaming
 * filter / channelizer objects compile unchanged against liquid-mi355x.
 */
#ifndef LIQUID_MI355X_COMPAT_LIQUID_H_TOP
#define LIQUID_MI355X_COMPAT_LIQUID_H_TOP
#include "liquid_mi355x.h"
#endif
