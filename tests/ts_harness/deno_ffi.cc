// deno_ffi.cc -- the part of Deno's FFI (Deno.dlopen, Deno.UnsafePointer, Deno.UnsafePointerView) that
// ts/verify.ts uses, as a Node 12 N-API addon.  Test infrastructure only: Deno is absent from the image, so
// the TypeScript binding runs under Node with this shim (tests/ts_harness/deno_shim.js) against the real
// libtorrent_verify.so.
//
//   open(path) -> handle (BigInt)          sym(handle, name) -> function address (BigInt)
//   call(fn, args: BigInt[] (<= 8, each the 64-bit register image of an integer / pointer argument),
//        result: 0 void | 1 i32) -> number | undefined
//   callAsync(fn, args, result) -> Promise of the same, the call run on a libuv worker thread
//   addressOf(typedArray) -> BigInt        arrayBuffer(address: BigInt, length) -> ArrayBuffer over it
//
// Every argument of the ABI is an integer or a pointer (include/torrent_verify.h), so on x86-64 System V
// they all travel in integer registers (the seventh on the stack): one call shape with seven 64-bit
// arguments serves every entry point (a callee with fewer parameters ignores the rest).
#include <dlfcn.h>
#include <node_api.h>
#include <stdint.h>
#include <string.h>

#include <string>

namespace {

napi_value throw_error(napi_env env, const std::string& msg) {
    napi_throw_error(env, nullptr, msg.c_str());
    return nullptr;
}

bool get_u64(napi_env env, napi_value v, uint64_t* out) {
    bool lossless = true;
    return napi_get_value_bigint_uint64(env, v, out, &lossless) == napi_ok;
}

napi_value make_u64(napi_env env, uint64_t v) {
    napi_value r;
    napi_create_bigint_uint64(env, v, &r);
    return r;
}

napi_value Open(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
    char path[4096];
    size_t n = 0;
    if (argc < 1 || napi_get_value_string_utf8(env, argv[0], path, sizeof path, &n) != napi_ok)
        return throw_error(env, "open(path): path must be a string");
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) return throw_error(env, std::string("dlopen failed: ") + dlerror());
    return make_u64(env, (uint64_t)(uintptr_t)h);
}

napi_value Sym(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
    uint64_t h = 0;
    char name[256];
    size_t n = 0;
    if (argc < 2 || !get_u64(env, argv[0], &h) || napi_get_value_string_utf8(env, argv[1], name, sizeof name, &n) != napi_ok)
        return throw_error(env, "sym(handle, name)");
    void* f = dlsym((void*)(uintptr_t)h, name);
    if (!f) return throw_error(env, std::string("dlsym failed: ") + name);
    return make_u64(env, (uint64_t)(uintptr_t)f);
}

typedef int64_t (*Fn8)(uint64_t, uint64_t, uint64_t, uint64_t, uint64_t, uint64_t, uint64_t, uint64_t);

napi_value Call(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
    uint64_t fn = 0;
    if (argc < 3 || !get_u64(env, argv[0], &fn)) return throw_error(env, "call(fn, args, result)");
    uint32_t nargs = 0;
    if (napi_get_array_length(env, argv[1], &nargs) != napi_ok || nargs > 8)
        return throw_error(env, "call: args must be an array of at most 8 BigInts");
    uint64_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t i = 0; i < nargs; i++) {
        napi_value e;
        napi_get_element(env, argv[1], i, &e);
        if (!get_u64(env, e, &a[i])) return throw_error(env, "call: every argument must be a BigInt");
    }
    int32_t kind = 0;
    napi_get_value_int32(env, argv[2], &kind);
    const int64_t r = ((Fn8)(uintptr_t)fn)(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7]);
    if (kind == 0) {
        napi_value u;
        napi_get_undefined(env, &u);
        return u;
    }
    napi_value out;
    napi_create_int32(env, (int32_t)r, &out);
    return out;
}

// callAsync: the same call on a libuv worker thread, returning a Promise -- Deno runs a `nonblocking` symbol
// on its blocking-task pool and resolves the promise on the event loop, so calls on different contexts
// really overlap, as they do under Deno.
struct AsyncCall {
    uint64_t fn;
    uint64_t a[8];
    int32_t kind;
    int64_t r;
    napi_deferred deferred;
    napi_async_work work;
};

void AsyncExecute(napi_env, void* data) {
    AsyncCall* c = (AsyncCall*)data;
    c->r = ((Fn8)(uintptr_t)c->fn)(c->a[0], c->a[1], c->a[2], c->a[3], c->a[4], c->a[5], c->a[6], c->a[7]);
}

void AsyncComplete(napi_env env, napi_status, void* data) {
    AsyncCall* c = (AsyncCall*)data;
    napi_value v;
    if (c->kind == 0) napi_get_undefined(env, &v);
    else napi_create_int32(env, (int32_t)c->r, &v);
    napi_resolve_deferred(env, c->deferred, v);
    napi_delete_async_work(env, c->work);
    delete c;
}

napi_value CallAsync(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
    AsyncCall* c = new AsyncCall();
    uint32_t nargs = 0;
    if (argc < 3 || !get_u64(env, argv[0], &c->fn) || napi_get_array_length(env, argv[1], &nargs) != napi_ok ||
        nargs > 8) {
        delete c;
        return throw_error(env, "callAsync(fn, args: at most 8 BigInts, result)");
    }
    for (uint32_t i = 0; i < nargs; i++) {
        napi_value e;
        napi_get_element(env, argv[1], i, &e);
        if (!get_u64(env, e, &c->a[i])) {
            delete c;
            return throw_error(env, "callAsync: every argument must be a BigInt");
        }
    }
    napi_get_value_int32(env, argv[2], &c->kind);
    napi_value promise, name;
    napi_create_promise(env, &c->deferred, &promise);
    napi_create_string_utf8(env, "deno_ffi_call", NAPI_AUTO_LENGTH, &name);
    napi_create_async_work(env, nullptr, name, AsyncExecute, AsyncComplete, c, &c->work);
    napi_queue_async_work(env, c->work);
    return promise;
}

napi_value AddressOf(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
    bool is_ta = false;
    napi_is_typedarray(env, argv[0], &is_ta);
    if (!is_ta) return throw_error(env, "addressOf: not a typed array");
    napi_typedarray_type type;
    size_t length, offset;
    void* data = nullptr;
    napi_value ab;
    napi_get_typedarray_info(env, argv[0], &type, &length, &data, &ab, &offset);
    return make_u64(env, (uint64_t)(uintptr_t)data);
}

napi_value ArrayBufferAt(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
    uint64_t p = 0;
    int64_t len = 0;
    if (argc < 2 || !get_u64(env, argv[0], &p) || napi_get_value_int64(env, argv[1], &len) != napi_ok || len < 0)
        return throw_error(env, "arrayBuffer(address, length)");
    napi_value ab;
    if (napi_create_external_arraybuffer(env, (void*)(uintptr_t)p, (size_t)len, nullptr, nullptr, &ab) != napi_ok)
        return throw_error(env, "napi_create_external_arraybuffer failed");
    return ab;
}

napi_value Init(napi_env env, napi_value exports) {
    const napi_property_descriptor props[] = {
        {"open", nullptr, Open, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"sym", nullptr, Sym, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"call", nullptr, Call, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"callAsync", nullptr, CallAsync, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"addressOf", nullptr, AddressOf, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"arrayBuffer", nullptr, ArrayBufferAt, nullptr, nullptr, nullptr, napi_default, nullptr},
    };
    napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
