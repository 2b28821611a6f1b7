/*
 * oracle/glsl_ref/display_harness.c — TEST INFRASTRUCTURE: runs the reference's display pass,
 * Graphics::Display (Graphics.cpp:356-390) with createFQ (Graphics.cpp:227-258) and the
 * FullQuad.vs / FullQuad.fs shader pair, headless on Mesa llvmpipe (DRI swrast, as harness.c).
 * The shader text is read from /root/reference at run time and never copied into the repo.
 *
 * GL state as the reference sets it: blending SRC_ALPHA / ONE_MINUS_SRC_ALPHA (Graphics.cpp:268-269),
 * GL_FRAMEBUFFER_SRGB on while drawing, the accumulator an RGBA32F texture with GL_NEAREST
 * (Graphics.h:85-91), uniforms tex / screenSize / bounds, one GL_QUADS draw of the four vertices
 * createFQ builds. The reference draws into the SFML window; here the target is an sRGB8_ALPHA8
 * texture of the screen size initialised with the caller's background (the GUI behind the image),
 * with the viewport covering it. The reference's compatibility context provides GL_QUADS; a
 * compatibility-profile 4.3 context is requested here too (a core context would lack it).
 *
 * usage: display_harness <FullQuad.vs> <FullQuad.fs> <accum.f32> W H <bg.rgba8> SW SH
 *                        CX CY ZOOM MINX MINY MAXX MAXY <out.rgba8>
 * out.rgba8: glReadPixels of the target, rows bottom-up (GL order).
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <GL/glcorearb.h>
#include <GL/internal/dri_interface.h>

#ifndef GL_QUADS
#define GL_QUADS 0x0007
#endif

static void gdi(__DRIdrawable* d, int* x, int* y, int* w, int* h, void* p) { (void)d; (void)p; *x = 0; *y = 0; *w = 1; *h = 1; }
static void pim(__DRIdrawable* d, int op, int x, int y, int w, int h, char* data, void* p) {
    (void)d; (void)op; (void)x; (void)y; (void)w; (void)h; (void)data; (void)p;
}
static void gim(__DRIdrawable* d, int x, int y, int w, int h, char* data, void* p) {
    (void)d; (void)x; (void)y; (void)w; (void)h; (void)data; (void)p;
}
static const __DRIswrastLoaderExtension loader = {{__DRI_SWRAST_LOADER, 1}, gdi, pim, gim, NULL, NULL};
static const __DRIextension* loader_exts[] = {&loader.base, NULL};

typedef void* (*getproc_t)(const char*);
static getproc_t getproc;
#define GLF(type, name) static type p_##name;
GLF(PFNGLCREATESHADERPROC, glCreateShader)
GLF(PFNGLSHADERSOURCEPROC, glShaderSource)
GLF(PFNGLCOMPILESHADERPROC, glCompileShader)
GLF(PFNGLGETSHADERIVPROC, glGetShaderiv)
GLF(PFNGLGETSHADERINFOLOGPROC, glGetShaderInfoLog)
GLF(PFNGLCREATEPROGRAMPROC, glCreateProgram)
GLF(PFNGLATTACHSHADERPROC, glAttachShader)
GLF(PFNGLLINKPROGRAMPROC, glLinkProgram)
GLF(PFNGLGETPROGRAMIVPROC, glGetProgramiv)
GLF(PFNGLGETPROGRAMINFOLOGPROC, glGetProgramInfoLog)
GLF(PFNGLUSEPROGRAMPROC, glUseProgram)
GLF(PFNGLGETUNIFORMLOCATIONPROC, glGetUniformLocation)
GLF(PFNGLUNIFORM1IPROC, glUniform1i)
GLF(PFNGLUNIFORM2FPROC, glUniform2f)
GLF(PFNGLUNIFORM4FPROC, glUniform4f)
GLF(PFNGLGENTEXTURESPROC, glGenTextures)
GLF(PFNGLBINDTEXTUREPROC, glBindTexture)
GLF(PFNGLACTIVETEXTUREPROC, glActiveTexture)
GLF(PFNGLTEXIMAGE2DPROC, glTexImage2D)
GLF(PFNGLTEXPARAMETERIPROC, glTexParameteri)
GLF(PFNGLGENFRAMEBUFFERSPROC, glGenFramebuffers)
GLF(PFNGLBINDFRAMEBUFFERPROC, glBindFramebuffer)
GLF(PFNGLFRAMEBUFFERTEXTURE2DPROC, glFramebufferTexture2D)
GLF(PFNGLCHECKFRAMEBUFFERSTATUSPROC, glCheckFramebufferStatus)
GLF(PFNGLVIEWPORTPROC, glViewport)
GLF(PFNGLENABLEPROC, glEnable)
GLF(PFNGLDISABLEPROC, glDisable)
GLF(PFNGLBLENDFUNCPROC, glBlendFunc)
GLF(PFNGLGENVERTEXARRAYSPROC, glGenVertexArrays)
GLF(PFNGLBINDVERTEXARRAYPROC, glBindVertexArray)
GLF(PFNGLGENBUFFERSPROC, glGenBuffers)
GLF(PFNGLBINDBUFFERPROC, glBindBuffer)
GLF(PFNGLBUFFERDATAPROC, glBufferData)
GLF(PFNGLENABLEVERTEXATTRIBARRAYPROC, glEnableVertexAttribArray)
GLF(PFNGLVERTEXATTRIBPOINTERPROC, glVertexAttribPointer)
GLF(PFNGLDRAWARRAYSPROC, glDrawArrays)
GLF(PFNGLFINISHPROC, glFinish)
GLF(PFNGLREADPIXELSPROC, glReadPixels)
GLF(PFNGLPIXELSTOREIPROC, glPixelStorei)
GLF(PFNGLGETERRORPROC, glGetError)
#define LOAD(name)                                                         \
    do {                                                                   \
        p_##name = (void*)getproc(#name);                                  \
        if (!p_##name) { fprintf(stderr, "missing %s\n", #name); exit(3); } \
    } while (0)

static char* slurp(const char* path, long* n) {
    FILE* f = fopen(path, "rb");
    if (!f) { perror(path); exit(2); }
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* b = malloc(sz + 1);
    if (fread(b, 1, sz, f) != (size_t)sz) { perror("read"); exit(2); }
    b[sz] = 0;
    fclose(f);
    if (n) *n = sz;
    return b;
}

/* texture2D( -> texture( : the same patch harness.c's callers apply to RayMarch*.glsl (Mesa rejects
 * texture2D under "#version 430 core") */
static char* patch_texture2d(char* src) {
    char* out = malloc(strlen(src) + 1);
    char* o = out;
    for (const char* s = src; *s;) {
        if (!strncmp(s, "texture2D(", 10)) { memcpy(o, "texture(", 8); o += 8; s += 10; }
        else *o++ = *s++;
    }
    *o = 0;
    return out;
}

static GLuint compile(GLenum type, const char* path) {
    char* src = patch_texture2d(slurp(path, NULL));
    GLuint sh = p_glCreateShader(type);
    p_glShaderSource(sh, 1, (const char* const*)&src, NULL);
    p_glCompileShader(sh);
    GLint ok = 0;
    p_glGetShaderiv(sh, GL_COMPILE_STATUS, &ok);
    if (!ok) {
        static char log[65536];
        p_glGetShaderInfoLog(sh, sizeof log, NULL, log);
        fprintf(stderr, "COMPILE ERROR %s\n%s\n", path, log);
        exit(4);
    }
    return sh;
}

int main(int argc, char** argv) {
    if (argc != 17) { fprintf(stderr, "usage: see display_harness.c\n"); return 1; }
    const int W = atoi(argv[4]), H = atoi(argv[5]), SW = atoi(argv[7]), SH = atoi(argv[8]);
    const float cx = strtof(argv[9], NULL), cy = strtof(argv[10], NULL), zoom = strtof(argv[11], NULL);
    const float bx0 = strtof(argv[12], NULL), by0 = strtof(argv[13], NULL);
    const float bx1 = strtof(argv[14], NULL), by1 = strtof(argv[15], NULL);

    void* glapi = dlopen("libglapi.so.0", RTLD_NOW | RTLD_GLOBAL);
    if (!glapi) { fprintf(stderr, "dlopen libglapi: %s\n", dlerror()); return 2; }
    const char* drvpath = getenv("RMR_SWRAST") ? getenv("RMR_SWRAST") : "/usr/lib/x86_64-linux-gnu/dri/swrast_dri.so";
    void* drv = dlopen(drvpath, RTLD_NOW | RTLD_GLOBAL);
    if (!drv) { fprintf(stderr, "dlopen swrast: %s\n", dlerror()); return 2; }
    const __DRIextension** (*getext)(void) = (const __DRIextension** (*)(void))dlsym(drv, "__driDriverGetExtensions_swrast");
    getproc = (getproc_t)dlsym(glapi, "_glapi_get_proc_address");
    if (!getext || !getproc) { fprintf(stderr, "missing driver entry points\n"); return 2; }
    const __DRIextension** ext = getext();
    const __DRIcoreExtension* core = NULL;
    const __DRIswrastExtension* sw = NULL;
    for (int i = 0; ext[i]; i++) {
        if (!strcmp(ext[i]->name, __DRI_CORE)) core = (const __DRIcoreExtension*)ext[i];
        if (!strcmp(ext[i]->name, __DRI_SWRAST)) sw = (const __DRIswrastExtension*)ext[i];
    }
    if (!core || !sw || sw->base.version < 4) { fprintf(stderr, "no DRI core/swrast v4\n"); return 2; }
    const __DRIconfig** cfgs = NULL;
    __DRIscreen* scr = sw->createNewScreen2(0, loader_exts, ext, &cfgs, NULL);
    if (!scr || !cfgs || !cfgs[0]) { fprintf(stderr, "createNewScreen2 failed\n"); return 2; }
    uint32_t attribs[] = {__DRI_CTX_ATTRIB_MAJOR_VERSION, 4, __DRI_CTX_ATTRIB_MINOR_VERSION, 3};
    unsigned err = 0;
    /* compatibility profile: GL_QUADS as the reference draws it */
    __DRIcontext* ctx = sw->createContextAttribs(scr, __DRI_API_OPENGL, cfgs[0], NULL, 2, attribs, &err, NULL);
    if (!ctx) { fprintf(stderr, "createContextAttribs (compat 4.3) failed (%u)\n", err); return 2; }
    if (!core->bindContext(ctx, NULL, NULL)) { fprintf(stderr, "bindContext failed\n"); return 2; }
    LOAD(glCreateShader); LOAD(glShaderSource); LOAD(glCompileShader); LOAD(glGetShaderiv);
    LOAD(glGetShaderInfoLog); LOAD(glCreateProgram); LOAD(glAttachShader); LOAD(glLinkProgram);
    LOAD(glGetProgramiv); LOAD(glGetProgramInfoLog); LOAD(glUseProgram); LOAD(glGetUniformLocation);
    LOAD(glUniform1i); LOAD(glUniform2f); LOAD(glUniform4f); LOAD(glGenTextures); LOAD(glBindTexture);
    LOAD(glActiveTexture); LOAD(glTexImage2D); LOAD(glTexParameteri); LOAD(glGenFramebuffers);
    LOAD(glBindFramebuffer); LOAD(glFramebufferTexture2D); LOAD(glCheckFramebufferStatus); LOAD(glViewport);
    LOAD(glEnable); LOAD(glDisable); LOAD(glBlendFunc); LOAD(glGenVertexArrays); LOAD(glBindVertexArray);
    LOAD(glGenBuffers); LOAD(glBindBuffer); LOAD(glBufferData); LOAD(glEnableVertexAttribArray);
    LOAD(glVertexAttribPointer); LOAD(glDrawArrays); LOAD(glFinish); LOAD(glReadPixels); LOAD(glPixelStorei);
    LOAD(glGetError);

    GLuint vs = compile(GL_VERTEX_SHADER, argv[1]), fs = compile(GL_FRAGMENT_SHADER, argv[2]);
    GLuint prog = p_glCreateProgram();
    p_glAttachShader(prog, vs);
    p_glAttachShader(prog, fs);
    p_glLinkProgram(prog);
    GLint ok = 0;
    p_glGetProgramiv(prog, GL_LINK_STATUS, &ok);
    if (!ok) {
        static char log[65536];
        p_glGetProgramInfoLog(prog, sizeof log, NULL, log);
        fprintf(stderr, "LINK ERROR\n%s\n", log);
        return 4;
    }

    /* the accumulator: Framebuffer::Create's RGBA32F texture, GL_NEAREST */
    long n = 0;
    float* acc = (float*)slurp(argv[3], &n);
    if (n != (long)W * H * 16) { fprintf(stderr, "accum size mismatch\n"); return 1; }
    GLuint tex = 0;
    p_glActiveTexture(GL_TEXTURE0);
    p_glGenTextures(1, &tex);
    p_glBindTexture(GL_TEXTURE_2D, tex);
    p_glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA32F, W, H, 0, GL_RGBA, GL_FLOAT, acc);
    p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MIN_FILTER, GL_NEAREST);
    p_glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MAG_FILTER, GL_NEAREST);

    /* the window: an sRGB-capable RGBA8 target holding the background, GL rows bottom-up */
    unsigned char* bg = (unsigned char*)slurp(argv[6], &n);
    if (n != (long)SW * SH * 4) { fprintf(stderr, "background size mismatch\n"); return 1; }
    GLuint target = 0, fbo = 0;
    p_glGenTextures(1, &target);
    p_glBindTexture(GL_TEXTURE_2D, target);
    p_glPixelStorei(GL_UNPACK_ALIGNMENT, 1);
    p_glTexImage2D(GL_TEXTURE_2D, 0, GL_SRGB8_ALPHA8, SW, SH, 0, GL_RGBA, GL_UNSIGNED_BYTE, bg);
    p_glGenFramebuffers(1, &fbo);
    p_glBindFramebuffer(GL_FRAMEBUFFER, fbo);
    p_glFramebufferTexture2D(GL_FRAMEBUFFER, GL_COLOR_ATTACHMENT0, GL_TEXTURE_2D, target, 0);
    if (p_glCheckFramebufferStatus(GL_FRAMEBUFFER) != GL_FRAMEBUFFER_COMPLETE) { fprintf(stderr, "fbo incomplete\n"); return 5; }
    p_glViewport(0, 0, SW, SH);

    /* Graphics::Init (Graphics.cpp:268-269) */
    p_glEnable(GL_BLEND);
    p_glBlendFunc(GL_SRC_ALPHA, GL_ONE_MINUS_SRC_ALPHA);

    /* Graphics::Display (Graphics.cpp:356-390) */
    p_glEnable(GL_FRAMEBUFFER_SRGB);
    p_glUseProgram(prog);
    p_glUniform1i(p_glGetUniformLocation(prog, "tex"), 0);
    p_glUniform2f(p_glGetUniformLocation(prog, "screenSize"), (float)SW, (float)SH);
    p_glUniform4f(p_glGetUniformLocation(prog, "bounds"), bx0, by0, bx1, by1);
    p_glActiveTexture(GL_TEXTURE0);
    p_glBindTexture(GL_TEXTURE_2D, tex);

    /* createFQ (Graphics.cpp:227-258): imageSize / 2 * zoom, vertices (pos.xy, uv.xy) */
    const float halfWidth = ((float)W / 2) * zoom;
    const float halfHeight = ((float)H / 2) * zoom;
    const GLfloat v[16] = {cx - halfWidth, cy - halfHeight, 0.0f, 0.0f,
                           cx + halfWidth, cy - halfHeight, 1.0f, 0.0f,
                           cx + halfWidth, cy + halfHeight, 1.0f, 1.0f,
                           cx - halfWidth, cy + halfHeight, 0.0f, 1.0f};
    GLuint vao = 0, vbo = 0;
    p_glGenVertexArrays(1, &vao);
    p_glBindVertexArray(vao);
    p_glGenBuffers(1, &vbo);
    p_glBindBuffer(GL_ARRAY_BUFFER, vbo);
    p_glBufferData(GL_ARRAY_BUFFER, sizeof v, v, GL_STATIC_DRAW);
    p_glEnableVertexAttribArray(0);
    p_glVertexAttribPointer(0, 2, GL_FLOAT, GL_FALSE, 4 * sizeof(GLfloat), 0);
    p_glEnableVertexAttribArray(1);
    p_glVertexAttribPointer(1, 2, GL_FLOAT, GL_FALSE, 4 * sizeof(GLfloat), (void*)(2 * sizeof(float)));
    p_glDrawArrays(GL_QUADS, 0, 4);
    p_glDisable(GL_FRAMEBUFFER_SRGB);
    p_glFinish();
    GLenum e = p_glGetError();
    if (e != GL_NO_ERROR) { fprintf(stderr, "GL error 0x%x\n", e); return 5; }

    unsigned char* out = malloc((size_t)SW * SH * 4);
    p_glPixelStorei(GL_PACK_ALIGNMENT, 1);
    p_glReadPixels(0, 0, SW, SH, GL_RGBA, GL_UNSIGNED_BYTE, out);
    FILE* f = fopen(argv[16], "wb");
    if (!f) { perror(argv[16]); return 2; }
    fwrite(out, 1, (size_t)SW * SH * 4, f);
    fclose(f);
    return 0;
}
