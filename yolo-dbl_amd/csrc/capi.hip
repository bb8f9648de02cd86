// Error plumbing and shared host-side validation for the C ABI.
#include "common.hpp"

namespace ydbl {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(YDBL_ELAUNCH, std::string(what) + ": " + hipGetErrorString(e));
  return YDBL_OK;
}

int check_view(const ydbl_view* v, const char* name, bool need_vec_align) {
  if (!v || !v->ptr) return fail(YDBL_EINVAL, std::string(name) + ": null view");
  if (v->dtype != YDBL_F32 && v->dtype != YDBL_F16) return fail(YDBL_EINVAL, std::string(name) + ": bad dtype");
  if (v->n < 1 || v->h < 1 || v->w < 1 || v->c < 1 || v->cs < v->c)
    return fail(YDBL_EINVAL, std::string(name) + ": bad shape");
  const int vec = v->dtype == YDBL_F16 ? 8 : 4;
  if (need_vec_align) {
    if (v->cs % vec || v->c % vec) return fail(YDBL_EINVAL, std::string(name) + ": channels not 16-byte aligned");
    if (reinterpret_cast<uintptr_t>(v->ptr) % 16) return fail(YDBL_EINVAL, std::string(name) + ": pointer not 16-byte aligned");
  }
  return YDBL_OK;
}

}  // namespace ydbl

extern "C" const char* ydbl_last_error(void) { return ydbl::g_last_error.c_str(); }
extern "C" const char* ydbl_version(void) { return "ydbl 0.1 gfx950"; }
