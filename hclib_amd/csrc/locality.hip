// locality.hip — modules, locale types, the locality graph and the host
// worker state of the HClib C API (host code; no kernels).
//
//   module registry + per-worker module state   src/hclib_module.c:49-160
//   module loading from `deps`                  src/hclib-runtime.c:294-317
//   locale types, initialize_locale, metadata   src/hclib-locality-graph.c:322-367
//   locality files (JSON)                       src/hclib-locality-graph.c:372-573
//   default graph                               src/hclib-locality-graph.c:581-643
//   locale queries                              src/hclib-locality-graph.c:829-1170
//   current_ws / ws_key / hclib_get_current_worker  src/hclib-runtime.c:73, 194-226
//
// This build's host has ONE worker (the control thread, worker 0); the GPU
// locales' workers are the megakernel's waves. A locality file's worker
// count is recorded (print_worker_paths shows every worker's paths) but only
// worker 0's paths are live. GPU-type locales map to HIP devices: the
// default graph has the process's bound GPU; a file's "GPU<k>" is device k.
#include <ctype.h>
#include <dlfcn.h>
#include <stdarg.h>
#include <stdint.h>
#include <string.h>

#include <memory>
#include <string>
#include <vector>

#include "hx_host.h"
#include "hx_module.h"

pthread_key_t ws_key;

namespace hxh {
namespace {

// ------------------------------------------------------------ modules
struct ModuleFns {
    std::string name;
    hclib_module_pre_init_func_type pre;
    hclib_module_post_init_func_type post;
    hclib_module_finalize_func_type fin;
};
std::vector<ModuleFns> &modules() {
    static std::vector<ModuleFns> m;
    return m;
}

// ------------------------------------------------------- locale types
std::vector<std::string> &types() {
    static std::vector<std::string> t{"sysmem"};  // kSysmemType; "GPU" comes from modules/hip
    return t;
}
struct MetaFns {
    hclib_locale_metadata_size_func_type size = nullptr;
    hclib_locale_metadata_populate_func_type populate = nullptr;
};
std::vector<MetaFns> &meta_fns() {
    static std::vector<MetaFns> m;
    return m;
}

// -------------------------------------------------------------- graph
struct Graph {
    bool built = false;
    hclib_locality_graph g{nullptr, 0, nullptr};
    std::vector<hclib_locale_t> locales;
    std::vector<unsigned> edges;
    std::vector<std::unique_ptr<char[]>> labels;
    std::vector<int> device;                    // per locale: GPU device or -1
    std::vector<std::vector<hclib_locale_t *>> pop, steal;  // per worker (file's count)
    std::vector<hclib_locality_path> pop_paths, steal_paths;
    std::vector<hclib_worker_paths> wpaths;
    int file_workers = 1;
    std::string source = "default";
};
Graph &graph() {
    static Graph G;
    return G;
}

hclib_worker_state g_ws0;
size_t g_module_state_size = 0;

const char *intern(const std::string &s) {
    Graph &G = graph();
    std::unique_ptr<char[]> p(new char[s.size() + 1]);
    memcpy(p.get(), s.c_str(), s.size() + 1);
    const char *r = p.get();
    G.labels.push_back(std::move(p));
    return r;
}

// initialize_locale, src/hclib-locality-graph.c:322-367: the first known
// type whose name is a prefix of the label; none is fatal
unsigned type_of_label(const std::string &lbl) {
    const std::vector<std::string> &t = types();
    for (size_t i = 0; i < t.size(); ++i)
        if (t[i].size() <= lbl.size() && lbl.compare(0, t[i].size(), t[i]) == 0) return (unsigned)i;
    fprintf(stderr, "Unknown locale type for locale \"%s\"\n", lbl.c_str());
    fprintf(stderr, "No module registered for these locales\n");
    exit(1);
}

int add_locale(const std::string &lbl) {
    Graph &G = graph();
    for (const hclib_locale_t &l : G.locales)
        if (lbl == l.lbl) die("locality graph: locale \"%s\" declared twice", lbl.c_str());
    hclib_locale_t l;
    memset(&l, 0, sizeof(l));
    l.id = (int)G.locales.size();
    l.type = type_of_label(lbl);
    l.lbl = intern(lbl);
    G.locales.push_back(l);
    G.device.push_back(-1);
    return l.id;
}

int find_locale(const std::string &lbl) {
    Graph &G = graph();
    for (const hclib_locale_t &l : G.locales)
        if (lbl == l.lbl) return l.id;
    return -1;
}

void finalize_graph(std::vector<std::pair<int, int>> &edges) {
    Graph &G = graph();
    const size_t n = G.locales.size();
    G.edges.assign(n * n, 0u);
    for (auto &e : edges) {
        G.edges[(size_t)e.first * n + e.second] = 1;
        G.edges[(size_t)e.second * n + e.first] = 1;
    }
    // GPU locales -> devices: "GPU<k>" is device k, otherwise the ordinal
    int ordinal = 0;
    for (size_t i = 0; i < n; ++i) {
        if (G.locales[i].type != gpu_type()) continue;
        const char *s = G.locales[i].lbl + 3;
        if (G.device[i] < 0) G.device[i] = (*s && isdigit((unsigned char)*s)) ? atoi(s) : ordinal;
        ordinal++;
    }
    // module metadata (src/hclib-locality-graph.c:356-366)
    for (hclib_locale_t &l : G.locales) {
        if (l.type < meta_fns().size() && meta_fns()[l.type].size) {
            l.metadata = malloc(meta_fns()[l.type].size());
            if (!l.metadata) die("out of memory");
            meta_fns()[l.type].populate(&l);
        }
    }
    G.g.locales = G.locales.data();
    G.g.n_locales = (unsigned)n;
    G.g.edges = G.edges.data();
    // worker paths
    const size_t nw = G.pop.size();
    G.pop_paths.resize(nw);
    G.steal_paths.resize(nw);
    G.wpaths.resize(nw);
    for (size_t w = 0; w < nw; ++w) {
        G.pop_paths[w] = {G.pop[w].data(), (unsigned)G.pop[w].size()};
        G.steal_paths[w] = {G.steal[w].data(), (unsigned)G.steal[w].size()};
        G.wpaths[w] = {&G.pop_paths[w], &G.steal_paths[w], 0};
    }
    // check_locality_graph, src/hclib-locality-graph.c:645-666
    for (hclib_locale_t &l : G.locales) l.reachable = 0;
    for (size_t w = 0; w < nw; ++w) {
        for (hclib_locale_t *l : G.pop[w]) l->reachable = 1;
        for (hclib_locale_t *l : G.steal[w]) l->reachable = 1;
    }
    g_ws0.paths = &G.wpaths[0];
    G.built = true;
}

// -------------------------------------------------- a small JSON reader
struct JVal {
    enum Kind { Null, Num, Str, Arr, Obj } kind = Null;
    double num = 0;
    std::string str;
    std::vector<JVal> items;                        // Arr
    std::vector<std::pair<std::string, JVal>> kv;   // Obj (file order)
    const JVal *get(const char *k) const {
        for (auto &p : kv)
            if (p.first == k) return &p.second;
        return nullptr;
    }
};

struct JParser {
    const char *p, *end;
    const char *file;
    [[noreturn]] void fail(const char *what) {
        fprintf(stderr, "Failed loading locality graph from %s: %s\n", file, what);
        exit(1);
    }
    void ws() {
        while (p < end && isspace((unsigned char)*p)) ++p;
    }
    std::string string() {
        if (*p != '"') fail("expected a string");
        std::string s;
        for (++p; p < end && *p != '"'; ++p) {
            if (*p == '\\' && p + 1 < end) ++p;
            s += *p;
        }
        if (p >= end) fail("unterminated string");
        ++p;
        return s;
    }
    JVal value() {
        ws();
        if (p >= end) fail("unexpected end of file");
        JVal v;
        if (*p == '{') {
            v.kind = JVal::Obj;
            ++p;
            ws();
            if (*p == '}') { ++p; return v; }
            while (true) {
                ws();
                std::string k = string();
                ws();
                if (*p != ':') fail("expected ':'");
                ++p;
                v.kv.emplace_back(k, value());
                ws();
                if (*p == ',') { ++p; continue; }
                if (*p == '}') { ++p; break; }
                fail("expected ',' or '}'");
            }
        } else if (*p == '[') {
            v.kind = JVal::Arr;
            ++p;
            ws();
            if (*p == ']') { ++p; return v; }
            while (true) {
                v.items.push_back(value());
                ws();
                if (*p == ',') { ++p; continue; }
                if (*p == ']') { ++p; break; }
                fail("expected ',' or ']'");
            }
        } else if (*p == '"') {
            v.kind = JVal::Str;
            v.str = string();
        } else {
            const char *s = p;
            while (p < end && (isalnum((unsigned char)*p) || *p == '-' || *p == '+' || *p == '.')) ++p;
            if (s == p) fail("unexpected character");
            std::string t(s, p);
            if (t == "null" || t == "true" || t == "false") return v;
            v.kind = JVal::Num;
            v.num = atof(t.c_str());
        }
        return v;
    }
};

// interpret_locale, src/hclib-locality-graph.c:150-236: "$(expr)" with
// operands `id` (the worker id) and integers, operators / and %, applied
// left to right
std::string interpret_label(const std::string &in, int wid, const char *file) {
    std::string out;
    size_t i = 0;
    auto skip = [&] { while (i < in.size() && in[i] == ' ') ++i; };
    auto operand = [&]() -> int {
        skip();
        if (in.compare(i, 2, "id") == 0) {
            i += 2;
            return wid;
        }
        size_t s = i;
        while (i < in.size() && isdigit((unsigned char)in[i])) ++i;
        if (s == i) {
            fprintf(stderr, "%s: bad operand in locale \"%s\"\n", file, in.c_str());
            exit(1);
        }
        return atoi(in.substr(s, i - s).c_str());
    };
    while (i < in.size()) {
        if (in[i] == '$' && i + 1 < in.size() && in[i + 1] == '(') {
            i += 2;
            int v = operand();
            skip();
            while (i < in.size() && in[i] != ')') {
                const char op = in[i++];
                const int r = operand();
                if (op == '/') v = r ? v / r : 0;
                else if (op == '%') v = r ? v % r : 0;
                else {
                    fprintf(stderr, "Unsupported op character \"%c\"\n", op);
                    exit(1);
                }
                skip();
            }
            ++i;  // ')'
            out += std::to_string(v);
        } else {
            out += in[i++];
        }
    }
    return out;
}

std::vector<hclib_locale_t *> parse_path(const JVal &arr, int wid, const char *file) {
    if (arr.kind != JVal::Arr || arr.items.empty()) {
        fprintf(stderr, "%s: a worker path must be a non-empty array of locales\n", file);
        exit(1);
    }
    std::vector<hclib_locale_t *> v;
    for (const JVal &s : arr.items) {
        if (s.kind != JVal::Str) die("%s: a path entry is not a string", file);
        const std::string lbl = interpret_label(s.str, wid, file);
        const int id = find_locale(lbl);
        if (id < 0) {
            fprintf(stderr, "failed finding locale to match lbl \"%s\"\n", lbl.c_str());
            exit(1);
        }
        v.push_back(&graph().locales[(size_t)id]);
    }
    return v;
}

void load_file(const char *file) {
    Graph &G = graph();
    FILE *fp = fopen(file, "rb");
    if (!fp) {
        fprintf(stderr, "Failed loading locality graph from %s\n", file);
        exit(1);
    }
    std::string text;
    char buf[4096];
    size_t k;
    while ((k = fread(buf, 1, sizeof(buf), fp)) > 0) text.append(buf, k);
    fclose(fp);
    JParser P{text.data(), text.data() + text.size(), file};
    const JVal root = P.value();
    if (root.kind != JVal::Obj) P.fail("the top level is not an object");
    const JVal *nw = root.get("nworkers"), *decl = root.get("declarations"),
               *reach = root.get("reachability"), *pops = root.get("pop_paths"),
               *steals = root.get("steal_paths");
    if (!nw || nw->kind != JVal::Num) P.fail("missing \"nworkers\"");
    if (!decl || decl->kind != JVal::Arr) P.fail("missing \"declarations\"");
    if (!reach || reach->kind != JVal::Arr) P.fail("missing \"reachability\"");
    if (!pops || pops->kind != JVal::Obj || !steals || steals->kind != JVal::Obj)
        P.fail("missing \"pop_paths\" / \"steal_paths\"");
    int nworkers = (int)nw->num;
    if (const char *e = getenv("HCLIB_WORKERS")) nworkers = atoi(e);
    if (nworkers < 1) nworkers = 1;
    G.file_workers = nworkers;
    G.locales.reserve(decl->items.size());
    for (const JVal &d : decl->items) {
        if (d.kind != JVal::Str) P.fail("a declaration is not a string");
        add_locale(d.str);
    }
    std::vector<std::pair<int, int>> edges;
    for (const JVal &e : reach->items) {
        if (e.kind != JVal::Arr || e.items.size() != 2 || e.items[0].kind != JVal::Str ||
            e.items[1].kind != JVal::Str)
            P.fail("a reachability edge is not a pair of locale names");
        const int a = find_locale(e.items[0].str), b = find_locale(e.items[1].str);
        if (a < 0 || b < 0) {
            fprintf(stderr, "Locale %s undeclared but referenced in reachability definition\n",
                    (a < 0 ? e.items[0] : e.items[1]).str.c_str());
            exit(1);
        }
        edges.emplace_back(a, b);
    }
    // per-worker paths: an entry keyed by the worker id, else "default"
    G.pop.resize((size_t)nworkers);
    G.steal.resize((size_t)nworkers);
    for (int w = 0; w < nworkers; ++w) {
        const std::string key = std::to_string(w);
        const JVal *pp = pops->get(key.c_str()) ? pops->get(key.c_str()) : pops->get("default");
        const JVal *sp = steals->get(key.c_str()) ? steals->get(key.c_str()) : steals->get("default");
        if (!pp || !sp) P.fail("no pop/steal path for a worker and no \"default\"");
        G.pop[(size_t)w] = parse_path(*pp, w, file);
        G.steal[(size_t)w] = parse_path(*sp, w, file);
    }
    G.source = file;
    finalize_graph(edges);
}

// the default graph of this build: system memory, the bound GPU (when the
// process sees one), and worker 0's private L1 locale when a module (the
// system module) has registered the L1 type, as the reference's default
// graph has one L1<i> per worker (src/hclib-locality-graph.c:608-637)
void build_default() {
    Graph &G = graph();
    std::vector<std::pair<int, int>> edges;
    G.locales.reserve(4);
    const int sys = add_locale("sysmem");
    int ndev = 0;
    if (gpu_type() != ~0u && hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    if (ndev > 0) {
        const int dev = hx::env_int("HCLIB_HIP_DEVICE", hx::env_int("LOCAL_RANK", 0));
        const int g = add_locale("GPU" + std::to_string(dev));
        G.device[(size_t)g] = dev;
        edges.emplace_back(sys, g);
    }
    int l1 = -1;
    for (size_t t = 0; t < types().size(); ++t)
        if (types()[t] == "L1") l1 = add_locale("L10");
    if (l1 >= 0) edges.emplace_back(sys, l1);
    G.pop.resize(1);
    G.steal.resize(1);
    if (l1 >= 0) {
        G.pop[0].push_back(&G.locales[(size_t)l1]);
        G.steal[0].push_back(&G.locales[(size_t)l1]);
    }
    G.pop[0].push_back(&G.locales[(size_t)sys]);
    G.steal[0].push_back(&G.locales[(size_t)sys]);
    finalize_graph(edges);
}

}  // namespace

void die(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    fprintf(stderr, "hclib: ");
    vfprintf(stderr, fmt, ap);
    fprintf(stderr, "\n");
    va_end(ap);
    abort();
}

// src/hclib-runtime.c:294-317. The directory: $HCLIB_MODULE_PATH, then
// $HCLIB_ROOT/lib (the reference's), then this library's own directory.
void load_dependencies(const char **deps, int ndeps) {
    std::vector<std::string> dirs;
    if (const char *mp = getenv("HCLIB_MODULE_PATH")) dirs.push_back(mp);
    if (const char *root = getenv("HCLIB_ROOT")) dirs.push_back(std::string(root) + "/lib");
    Dl_info info;
    if (dladdr((void *)&load_dependencies, &info) && info.dli_fname) {
        std::string self = info.dli_fname;
        const size_t slash = self.rfind('/');
        if (slash != std::string::npos) dirs.push_back(self.substr(0, slash));
    }
    for (int i = 0; i < ndeps; ++i) {
        const std::string name = deps[i];
        void *h = nullptr;
        std::string tried;
        for (const std::string &d : dirs) {
            const std::string path = d + "/libhclib_" + name + ".so";
            h = dlopen(path.c_str(), RTLD_LAZY | RTLD_GLOBAL);
            if (h) break;
            tried = path;
        }
        // "system": the host's system memory locale and its callbacks are
        // built in, so the module library is optional
        if (!h && name != "system")
            fprintf(stderr, "WARNING: Failed dynamically loading %s for \"%s\" dependency: %s\n",
                    tried.c_str(), name.c_str(), dlerror());
    }
}

namespace {
void prepare() {
    static bool done = false;
    if (done) return;
    if (pthread_key_create(&ws_key, nullptr) != 0) die("cannot create ws_key");
    g_ws0.id = 0;
    g_ws0.nworkers = 1;
    done = true;
}
}  // namespace

void build_graph() {
    if (graph().built) return;
    prepare();
    const char *file = getenv("HCLIB_LOCALITY_FILE");
    if (file && *file) load_file(file);
    else build_default();
}

int locale_device(const hclib_locale_t *l) {
    Graph &G = graph();
    if (!l || l->type != gpu_type()) return -1;
    const ptrdiff_t i = l - G.locales.data();
    if (i < 0 || (size_t)i >= G.locales.size()) return -1;
    return G.device[(size_t)i];
}

unsigned gpu_type() {
    const std::vector<std::string> &t = types();
    for (size_t i = 0; i < t.size(); ++i)
        if (t[i] == "GPU") return (unsigned)i;
    return ~0u;
}

hclib_worker_state *worker0() { return &g_ws0; }

void bind_worker0() {
    build_graph();
    pthread_setspecific(ws_key, &g_ws0);
}

}  // namespace hxh

using namespace hxh;

extern "C" {

// ------------------------------------------------------------ modules
// src/hclib_module.c:49-76: registering the same functions twice is a no-op
int hclib_add_module_init_function(const char *lbl, hclib_module_pre_init_func_type pre,
                                   hclib_module_post_init_func_type post,
                                   hclib_module_finalize_func_type finalize) {
    for (const ModuleFns &m : modules())
        if (m.pre == pre && m.post == post && m.fin == finalize) return 0;
    modules().push_back(ModuleFns{lbl ? lbl : "", pre, post, finalize});
    return 0;
}

void hclib_call_module_pre_init_functions(void) {
    for (size_t i = 0; i < modules().size(); ++i)
        if (modules()[i].pre) modules()[i].pre();
}
void hclib_call_module_post_init_functions(void) {
    for (size_t i = 0; i < modules().size(); ++i)
        if (modules()[i].post) modules()[i].post();
}
void hclib_call_finalize_functions(void) {
    for (size_t i = 0; i < modules().size(); ++i)
        if (modules()[i].fin) modules()[i].fin();
}

void hclib_add_locale_metadata_functions(int locale_id, hclib_locale_metadata_size_func_type size_func,
                                         hclib_locale_metadata_populate_func_type populate_func) {
    if (locale_id < 0 || !size_func || !populate_func) die("hclib_add_locale_metadata_functions: bad arguments");
    if (meta_fns().size() <= (size_t)locale_id) meta_fns().resize((size_t)locale_id + 1);
    meta_fns()[(size_t)locale_id] = MetaFns{size_func, populate_func};
}

// src/hclib_module.c:129-160 over this build's host workers (worker 0)
unsigned hclib_add_per_worker_module_state(size_t state_size, hclib_state_adder cb, void *user_data) {
    const unsigned offset = (unsigned)g_module_state_size;
    g_ws0.module_state = (char *)realloc(g_ws0.module_state, g_module_state_size + state_size);
    if (!g_ws0.module_state) die("out of memory");
    if (cb) cb(g_ws0.module_state + offset, user_data, 0);
    g_module_state_size += state_size;
    return offset;
}

void *hclib_get_curr_worker_module_state(const unsigned state_id) {
    hclib_worker_state *ws = current_ws();
    if (!ws || !ws->module_state || state_id >= g_module_state_size)
        die("hclib_get_curr_worker_module_state: no state %u on this thread", state_id);
    return ws->module_state + state_id;
}

void hclib_release_per_worker_module_state(const unsigned state_id, hclib_state_releaser cb, void *user_data) {
    if (!g_ws0.module_state || state_id >= g_module_state_size)
        die("hclib_release_per_worker_module_state: no state %u", state_id);
    if (cb) cb(g_ws0.module_state + state_id, user_data);
}

// ------------------------------------------------------ worker state
hclib_worker_state *current_ws(void) {
    build_graph();
    return (hclib_worker_state *)pthread_getspecific(ws_key);
}

int hclib_get_current_worker(void) {
    hclib_worker_state *ws = current_ws();
    if (!ws) die("hclib_get_current_worker called from a thread that is not an hclib worker");
    return ws->id;
}

int hclib_get_num_workers(void) { return 1; }

// ------------------------------------------------------- locale types
unsigned hclib_add_known_locale_type(const char *lbl) {
    std::vector<std::string> &t = types();
    for (size_t i = 0; i < t.size(); ++i)
        if (t[i] == lbl) return (unsigned)i;
    t.push_back(lbl);
    return (unsigned)t.size() - 1;
}

int hclib_get_locale_type(hclib_locale_t *l) {
    if (!l) die("hclib_get_locale_type: NULL locale");
    return (int)l->type;
}

const char *hclib_get_locale_type_name(int type) {
    return (type >= 0 && type < (int)types().size()) ? types()[(size_t)type].c_str() : nullptr;
}

// -------------------------------------------------------------- graph
void load_locality_info(const char *filename, int *nworkers_out, hclib_locality_graph **graph_out,
                        hclib_worker_paths **worker_paths_out) {
    Graph &G = graph();
    if (G.built) die("load_locality_info: the locality graph is already built (from %s)", G.source.c_str());
    prepare();
    load_file(filename);
    if (nworkers_out) *nworkers_out = G.file_workers;
    if (graph_out) *graph_out = &G.g;
    if (worker_paths_out) *worker_paths_out = G.wpaths.data();
}

void generate_locality_info(int *nworkers_out, hclib_locality_graph **graph_out,
                            hclib_worker_paths **worker_paths_out) {
    build_graph();
    Graph &G = graph();
    if (nworkers_out) *nworkers_out = G.file_workers;
    if (graph_out) *graph_out = &G.g;
    if (worker_paths_out) *worker_paths_out = G.wpaths.data();
}

void print_locality_graph(hclib_locality_graph *g) {
    fprintf(stderr, "==========================================\n");
    fprintf(stderr, "Locality graph (%u locales)\n", g->n_locales);
    for (unsigned i = 0; i < g->n_locales; ++i) {
        fprintf(stderr, "  %s (type %s):", g->locales[i].lbl, hclib_get_locale_type_name((int)g->locales[i].type));
        for (unsigned j = 0; j < g->n_locales; ++j)
            if (g->edges[i * g->n_locales + j]) fprintf(stderr, " %s", g->locales[j].lbl);
        fprintf(stderr, "\n");
    }
    fprintf(stderr, "==========================================\n");
}

void print_worker_paths(hclib_worker_paths *paths, int nworkers) {
    for (int w = 0; w < nworkers; ++w) {
        fprintf(stderr, "Worker %d\n  pop path:", w);
        for (unsigned j = 0; j < paths[w].pop_path->path_length; ++j)
            fprintf(stderr, " %s", paths[w].pop_path->locales[j]->lbl);
        fprintf(stderr, "\n  steal path:");
        for (unsigned j = 0; j < paths[w].steal_path->path_length; ++j)
            fprintf(stderr, " %s", paths[w].steal_path->locales[j]->lbl);
        fprintf(stderr, "\n");
    }
}

int hclib_get_num_locales(void) {
    build_graph();
    return (int)graph().locales.size();
}

hclib_locale_t *hclib_get_all_locales(void) {
    build_graph();
    return graph().locales.data();
}

hclib_locale_t *hclib_get_locale(int index) {
    build_graph();
    Graph &G = graph();
    return (index >= 0 && (size_t)index < G.locales.size()) ? &G.locales[(size_t)index] : nullptr;
}

hclib_locale_t **hclib_get_all_locales_of_type(int type, int *out_count) {
    build_graph();
    Graph &G = graph();
    hclib_locale_t **v = (hclib_locale_t **)malloc(sizeof(hclib_locale_t *) * (G.locales.size() + 1));
    if (!v) die("out of memory");
    int k = 0;
    for (hclib_locale_t &l : G.locales)
        if ((int)l.type == type) v[k++] = &l;
    if (out_count) *out_count = k;
    return v;
}

int hclib_get_num_locales_of_type(int type) {
    build_graph();
    int n = 0;
    for (hclib_locale_t &l : graph().locales) n += (int)l.type == type;
    return n;
}

// breadth-first from `locale` over the reachability edges
// (src/hclib-locality-graph.c:1136-1165)
hclib_locale_t *hclib_get_closest_locale_of_types(hclib_locale_t *locale, int *locale_types, int n_locale_types) {
    build_graph();
    Graph &G = graph();
    const size_t n = G.locales.size();
    if (!locale || locale < G.locales.data() || locale >= G.locales.data() + n)
        die("hclib_get_closest_locale_of_types: not a locale of this graph");
    std::vector<int> q{locale->id};
    std::vector<char> seen(n, 0);
    seen[(size_t)locale->id] = 1;
    for (size_t h = 0; h < q.size(); ++h) {
        hclib_locale_t *cur = &G.locales[(size_t)q[h]];
        for (int t = 0; t < n_locale_types; ++t)
            if ((int)cur->type == locale_types[t]) return cur;
        for (size_t j = 0; j < n; ++j)
            if (G.edges[(size_t)cur->id * n + j] && !seen[j]) {
                seen[j] = 1;
                q.push_back((int)j);
            }
    }
    return nullptr;
}

hclib_locale_t *hclib_get_closest_locale_of_type(hclib_locale_t *locale, int type) {
    return hclib_get_closest_locale_of_types(locale, &type, 1);
}

// src/hclib-locality-graph.c:901-903: the first locale of the caller's pop path
hclib_locale_t *hclib_get_closest_locale(void) {
    build_graph();
    hclib_worker_state *ws = (hclib_worker_state *)pthread_getspecific(ws_key);
    if (!ws) ws = &g_ws0;  // a thread outside hclib_launch: worker 0's view
    return ws->paths->pop_path->locales[0];
}

// src/hclib-locality-graph.c:1020-1022
hclib_locale_t *hclib_get_master_place(void) {
    build_graph();
    return g_ws0.paths->pop_path->locales[0];
}

// src/hclib-locality-graph.c:1056-1100: the first locale of worker 0's steal
// path that is on its pop path and on every other worker's pop and steal
// paths (every worker the graph declares)
hclib_locale_t *hclib_get_central_place(void) {
    build_graph();
    Graph &G = graph();
    for (hclib_locale_t *c : G.steal[0]) {
        bool everywhere = true;
        for (size_t w = 0; w < G.pop.size() && everywhere; ++w) {
            bool in_pop = false, in_steal = false;
            for (hclib_locale_t *p : G.pop[w]) in_pop |= p == c;
            for (hclib_locale_t *p : G.steal[w]) in_steal |= p == c;
            everywhere = in_pop && in_steal;
        }
        if (everywhere) return c;
    }
    return nullptr;
}

// src/hclib-locality-graph.c:917-1017: per live worker, the earliest locale
// of its steal path that is also on its pop path, on no other worker's
// paths (every worker the file declares counts) and not marked special
hclib_locale_t **hclib_get_thread_private_locales(void) {
    build_graph();
    Graph &G = graph();
    hclib_locale_t **v = (hclib_locale_t **)malloc(sizeof(hclib_locale_t *));
    if (!v) die("out of memory");
    v[0] = nullptr;
    for (hclib_locale_t *c : G.steal[0]) {
        bool in_pop = false, elsewhere = false;
        for (hclib_locale_t *p : G.pop[0]) in_pop |= p == c;
        for (size_t w = 1; w < G.pop.size() && !elsewhere; ++w) {
            for (hclib_locale_t *p : G.pop[w]) elsewhere |= p == c;
            for (hclib_locale_t *p : G.steal[w]) elsewhere |= p == c;
        }
        if (in_pop && !elsewhere && !c->special_type) {
            v[0] = c;
            break;
        }
    }
    return v;
}

// src/hclib-locality-graph.c:829-837
void hclib_locale_mark_special(hclib_locale_t *locale, const char *special_type) {
    if (!locale || !special_type) die("hclib_locale_mark_special: null argument");
    if (locale->special_type) {
        if (strcmp(locale->special_type, special_type) != 0)
            die("hclib_locale_mark_special: locale already marked '%s'", locale->special_type);
    } else {
        locale->special_type = special_type;
    }
}

}  // extern "C"
