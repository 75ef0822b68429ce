/*
 * jni_mock.c — TEST INFRASTRUCTURE ONLY (tests/test_jni_shim.py).  A minimal
 * JNIEnv for exercising jni/HipNative.c without a JVM: the function-table
 * entries the shim calls, over plain C objects (direct buffers, int / float
 * arrays, strings, classes), and a pending-exception slot that ThrowNew
 * fills.  Linked with HipNative.c and librtamd.so into libhipnative_mock.so;
 * Python drives it through ctypes as the JVM would drive the shim.
 */
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { K_CLASS = 1, K_DIRECT, K_INTS, K_FLOATS, K_STRING };

struct mock_jobject {
    int kind;
    void* data;        /* buffer address, array elements, C string, class name */
    jlong n;           /* capacity in bytes / elements */
};

#define CHECK_INDEX(field, idx) \
    _Static_assert(offsetof(struct JNINativeInterface_, field) == (idx) * sizeof(void*), #field " index")
CHECK_INDEX(FindClass, 6);
CHECK_INDEX(ThrowNew, 14);
CHECK_INDEX(ExceptionOccurred, 15);
CHECK_INDEX(ExceptionClear, 17);
CHECK_INDEX(NewStringUTF, 167);
CHECK_INDEX(GetStringUTFChars, 169);
CHECK_INDEX(ReleaseStringUTFChars, 170);
CHECK_INDEX(GetArrayLength, 171);
CHECK_INDEX(GetIntArrayElements, 187);
CHECK_INDEX(GetFloatArrayElements, 189);
CHECK_INDEX(ReleaseIntArrayElements, 195);
CHECK_INDEX(ReleaseFloatArrayElements, 197);
CHECK_INDEX(ExceptionCheck, 228);
CHECK_INDEX(NewDirectByteBuffer, 229);
CHECK_INDEX(GetDirectBufferAddress, 230);
CHECK_INDEX(GetDirectBufferCapacity, 231);

static char g_ex_class[256];
static char g_ex_msg[2048];
static int g_ex_pending = 0;
static int g_outstanding = 0;          /* Get*Elements / GetStringUTFChars not yet released */

static jobject mk(int kind, void* data, jlong n) {
    struct mock_jobject* o = (struct mock_jobject*)calloc(1, sizeof *o);
    o->kind = kind;
    o->data = data;
    o->n = n;
    return o;
}

static jclass JNICALL FindClass(JNIEnv* env, const char* name) {
    (void)env;
    return mk(K_CLASS, strdup(name), 0);
}
static jint JNICALL ThrowNew(JNIEnv* env, jclass c, const char* msg) {
    (void)env;
    strncpy(g_ex_class, c && c->kind == K_CLASS ? (const char*)c->data : "?", sizeof g_ex_class - 1);
    strncpy(g_ex_msg, msg ? msg : "", sizeof g_ex_msg - 1);
    g_ex_pending = 1;
    return 0;
}
static jthrowable JNICALL ExceptionOccurred(JNIEnv* env) { (void)env; return g_ex_pending ? mk(K_CLASS, g_ex_class, 0) : NULL; }
static void JNICALL ExceptionClear(JNIEnv* env) { (void)env; g_ex_pending = 0; }
static jboolean JNICALL ExceptionCheck(JNIEnv* env) { (void)env; return (jboolean)g_ex_pending; }
static jstring JNICALL NewStringUTF(JNIEnv* env, const char* s) { (void)env; return mk(K_STRING, strdup(s), (jlong)strlen(s)); }
static const char* JNICALL GetStringUTFChars(JNIEnv* env, jstring s, jboolean* copy) {
    (void)env;
    if (copy) *copy = JNI_FALSE;
    ++g_outstanding;
    return (const char*)s->data;
}
static void JNICALL ReleaseStringUTFChars(JNIEnv* env, jstring s, const char* p) { (void)env; (void)s; (void)p; --g_outstanding; }
static jsize JNICALL GetArrayLength(JNIEnv* env, jarray a) { (void)env; return (jsize)a->n; }
static jint* JNICALL GetIntArrayElements(JNIEnv* env, jintArray a, jboolean* copy) {
    (void)env;
    if (copy) *copy = JNI_FALSE;
    ++g_outstanding;
    return a->kind == K_INTS ? (jint*)a->data : NULL;
}
static jfloat* JNICALL GetFloatArrayElements(JNIEnv* env, jfloatArray a, jboolean* copy) {
    (void)env;
    if (copy) *copy = JNI_FALSE;
    ++g_outstanding;
    return a->kind == K_FLOATS ? (jfloat*)a->data : NULL;
}
static void JNICALL ReleaseIntArrayElements(JNIEnv* env, jintArray a, jint* p, jint mode) {
    (void)env; (void)a; (void)p; (void)mode; --g_outstanding;
}
static void JNICALL ReleaseFloatArrayElements(JNIEnv* env, jfloatArray a, jfloat* p, jint mode) {
    (void)env; (void)a; (void)p; (void)mode; --g_outstanding;
}
static jobject JNICALL NewDirectByteBuffer(JNIEnv* env, void* p, jlong cap) { (void)env; return mk(K_DIRECT, p, cap); }
static void* JNICALL GetDirectBufferAddress(JNIEnv* env, jobject b) {
    (void)env;
    return b && b->kind == K_DIRECT ? b->data : NULL;        /* NULL for a non-direct buffer, as the JVM */
}
static jlong JNICALL GetDirectBufferCapacity(JNIEnv* env, jobject b) { (void)env; return b && b->kind == K_DIRECT ? b->n : -1; }

static struct JNINativeInterface_ g_table;
static JNIEnv g_env = &g_table;

/* ---- the harness side (ctypes) ---------------------------------------- */

JNIEnv* mock_env(void) {
    memset(&g_table, 0, sizeof g_table);      /* every other entry: NULL (a call would fault the test) */
    g_table.FindClass = FindClass;
    g_table.ThrowNew = ThrowNew;
    g_table.ExceptionOccurred = ExceptionOccurred;
    g_table.ExceptionClear = ExceptionClear;
    g_table.ExceptionCheck = ExceptionCheck;
    g_table.NewStringUTF = NewStringUTF;
    g_table.GetStringUTFChars = GetStringUTFChars;
    g_table.ReleaseStringUTFChars = ReleaseStringUTFChars;
    g_table.GetArrayLength = GetArrayLength;
    g_table.GetIntArrayElements = GetIntArrayElements;
    g_table.GetFloatArrayElements = GetFloatArrayElements;
    g_table.ReleaseIntArrayElements = ReleaseIntArrayElements;
    g_table.ReleaseFloatArrayElements = ReleaseFloatArrayElements;
    g_table.NewDirectByteBuffer = NewDirectByteBuffer;
    g_table.GetDirectBufferAddress = GetDirectBufferAddress;
    g_table.GetDirectBufferCapacity = GetDirectBufferCapacity;
    g_ex_pending = 0;
    g_outstanding = 0;
    return &g_env;
}
jobject mock_direct_buffer(void* p, jlong cap) { return mk(K_DIRECT, p, cap); }
jobject mock_heap_buffer(void) { return mk(K_CLASS, (void*)"java/nio/HeapByteBuffer", 0); }
jobject mock_int_array(jint* p, jsize n) { return mk(K_INTS, p, n); }
jobject mock_float_array(jfloat* p, jsize n) { return mk(K_FLOATS, p, n); }
jobject mock_string(const char* s) { return mk(K_STRING, strdup(s), (jlong)strlen(s)); }
void* mock_buffer_address(jobject b) { return b && b->kind == K_DIRECT ? b->data : NULL; }
jlong mock_buffer_capacity(jobject b) { return b && b->kind == K_DIRECT ? b->n : -1; }
int mock_outstanding(void) { return g_outstanding; }
/* 1 and the exception's class and message if one is pending (then cleared). */
int mock_take_exception(char* cls, size_t ncls, char* msg, size_t nmsg) {
    if (!g_ex_pending) return 0;
    strncpy(cls, g_ex_class, ncls - 1);
    cls[ncls - 1] = 0;
    strncpy(msg, g_ex_msg, nmsg - 1);
    msg[nmsg - 1] = 0;
    g_ex_pending = 0;
    return 1;
}
