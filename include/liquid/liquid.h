/*
 * liquid/liquid.h -- drop-in include path: programs written for liquid-dsp
 * (`#include <liquid/liquid.h>`) that use only the streaming filter /
 * channelizer objects compile unchanged against liquid-mi355x.
 */
#ifndef LIQUID_MI355X_COMPAT_LIQUID_H
#define LIQUID_MI355X_COMPAT_LIQUID_H
#include "../liquid_mi355x.h"
#endif
