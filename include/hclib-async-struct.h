/*
 * hclib-async-struct.h — task-record spawn entry points (MI355X build).
 *
 * The reference's header-only C++ layer builds an hclib_task_t itself and
 * hands it to these (inc/hclib-async-struct.h:49-54; callers
 * inc/hclib-async.h:153-290). Semantics of src/hclib-runtime.c:572-644
 * (spawn_handler): the task checks in on the caller's current finish, its
 * futures are copied into waiting_on[] (extras into a NULL-terminated
 * waiting_on_extra), and it is scheduled once every future is satisfied.
 * The runtime owns the record from here on and frees it after it ran.
 */
#ifndef HCLIB_ASYNCSTRUCT_H_
#define HCLIB_ASYNCSTRUCT_H_

#include <string.h>

#include "hclib-task.h"

#ifdef __cplusplus
extern "C" {
#endif

extern void spawn(hclib_task_t *task);
extern void spawn_await_at(hclib_task_t *task, hclib_future_t **futures, const int nfutures,
                           hclib_locale_t *locale);
extern void spawn_at(hclib_task_t *task, hclib_locale_t *locale);
extern void spawn_await(hclib_task_t *task, hclib_future_t **futures, const int nfutures);

#ifdef __cplusplus
}
#endif

#endif /* HCLIB_ASYNCSTRUCT_H_ */
