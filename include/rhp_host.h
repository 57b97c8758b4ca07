/*
 * rhp_host.h -- host-side entry points of librhp_host.so (no GPU).
 *
 *   rhp_cpu_parse_batch   the product's exact scalar parser (rhp_scalar.h, the
 *                         same code the kernel's rare paths run) over a batch in
 *                         host memory; the reactor's http_read_request and its
 *                         "host" session parser use it
 *   rhp_emu_parse_batch   CPU emulation of the kernel's DFA algorithm, block for
 *                         block (tests only); stats[3] = fast ok, fast -1, exact
 *
 * Both take an rhp_batch_t (include/rhp.h) whose pointers are host memory.
 */
#ifndef RHP_HOST_H
#define RHP_HOST_H

#include <stdint.h>
#include "rhp.h"

#ifdef __cplusplus
extern "C" {
#endif

int rhp_cpu_parse_batch(const rhp_batch_t *batch);
int rhp_emu_parse_batch(const rhp_batch_t *batch, uint64_t *stats);

#ifdef __cplusplus
}
#endif
#endif
