/*
 * hclib_common.h — default async arguments (inc/hclib_common.h:10-22).
 * The reference also includes its CMake-generated hclib_config.h here; this
 * build has no configure step, so there is nothing to include.
 */
#ifndef HCLIB_COMMON_H_
#define HCLIB_COMMON_H_

#define NO_PROP 0
#define NO_ARG NULL
#define NO_DATUM NULL
#define NO_FUTURE NULL
#define ANY_PLACE NULL
#define NO_ACCUM NULL

#endif
