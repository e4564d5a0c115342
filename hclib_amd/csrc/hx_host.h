// hx_host.h — host half of the HClib C API shared between hclib_api.hip
// (tasks, finish, promises, memory at locales) and locality.hip (modules,
// locale types, the locality graph, worker state).
#pragma once

#include "../../include/hclib.h"

namespace hxh {

[[noreturn]] void die(const char *fmt, ...);

// ---- modules (src/hclib_module.c:49-160, src/hclib-runtime.c:294-317)
// dlopen libhclib_<dep>.so for each dep ("hip" is this project's
// libhclib_hip.so plug-in, hclib_amd/csrc/modules/); the library's
// HCLIB_REGISTER_MODULE runs in its static initialiser
void load_dependencies(const char **deps, int ndeps);

// ---- locale types and the graph (src/hclib-locality-graph.c)
constexpr unsigned kSysmemType = 0;  // built in: system memory
// the "GPU" locale type once a module (modules/hip) has registered it, else
// an id no locale has
unsigned gpu_type();
// build the graph once the modules' pre-init functions have run
// (HCLIB_LOCALITY_FILE or the default graph); idempotent
void build_graph();
// the GPU device a GPU-type locale stands for (-1 for other locales)
int locale_device(const hclib_locale_t *l);
// worker 0 = the host control thread (the only host worker of this build)
hclib_worker_state *worker0();
void bind_worker0();  // make current_ws()/ws_key answer on the calling thread

}  // namespace hxh
