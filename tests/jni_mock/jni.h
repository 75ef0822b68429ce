/*
 * jni.h — TEST INFRASTRUCTURE ONLY (tests/test_jni_shim.py).  This image has
 * no JDK, so jni/HipNative.c is compiled for its test against this minimal
 * header: the JNI primitive and reference types and the JNIEnv function
 * table laid out by the indices of the JNI specification ("Interface
 * Function Table": FindClass 6, ThrowNew 14, GetStringUTFChars 169,
 * GetArrayLength 171, GetIntArrayElements 187, GetFloatArrayElements 189,
 * ReleaseIntArrayElements 195, ReleaseFloatArrayElements 197,
 * NewDirectByteBuffer 229, GetDirectBufferAddress 230, ...).  Only the
 * entries the shim (and the mock) use are typed; the rest are placeholders,
 * so a call to any other entry would be a test failure, not silent.
 * tests/jni_mock/jni_mock.c checks the typed entries' offsets against those
 * indices at compile time.
 */
#ifndef RTAMD_TEST_JNI_H
#define RTAMD_TEST_JNI_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_COMMIT 1
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

typedef struct mock_jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jintArray;
typedef jarray jfloatArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
    void* unused_0;
    void* unused_1;
    void* unused_2;
    void* unused_3;
    void* unused_4;
    void* unused_5;
    jclass (JNICALL *FindClass)(JNIEnv*, const char*);  /* 6 */
    void* unused_7;
    void* unused_8;
    void* unused_9;
    void* unused_10;
    void* unused_11;
    void* unused_12;
    void* unused_13;
    jint (JNICALL *ThrowNew)(JNIEnv*, jclass, const char*);  /* 14 */
    jthrowable (JNICALL *ExceptionOccurred)(JNIEnv*);  /* 15 */
    void* unused_16;
    void (JNICALL *ExceptionClear)(JNIEnv*);  /* 17 */
    void* unused_18;
    void* unused_19;
    void* unused_20;
    void* unused_21;
    void* unused_22;
    void* unused_23;
    void* unused_24;
    void* unused_25;
    void* unused_26;
    void* unused_27;
    void* unused_28;
    void* unused_29;
    void* unused_30;
    void* unused_31;
    void* unused_32;
    void* unused_33;
    void* unused_34;
    void* unused_35;
    void* unused_36;
    void* unused_37;
    void* unused_38;
    void* unused_39;
    void* unused_40;
    void* unused_41;
    void* unused_42;
    void* unused_43;
    void* unused_44;
    void* unused_45;
    void* unused_46;
    void* unused_47;
    void* unused_48;
    void* unused_49;
    void* unused_50;
    void* unused_51;
    void* unused_52;
    void* unused_53;
    void* unused_54;
    void* unused_55;
    void* unused_56;
    void* unused_57;
    void* unused_58;
    void* unused_59;
    void* unused_60;
    void* unused_61;
    void* unused_62;
    void* unused_63;
    void* unused_64;
    void* unused_65;
    void* unused_66;
    void* unused_67;
    void* unused_68;
    void* unused_69;
    void* unused_70;
    void* unused_71;
    void* unused_72;
    void* unused_73;
    void* unused_74;
    void* unused_75;
    void* unused_76;
    void* unused_77;
    void* unused_78;
    void* unused_79;
    void* unused_80;
    void* unused_81;
    void* unused_82;
    void* unused_83;
    void* unused_84;
    void* unused_85;
    void* unused_86;
    void* unused_87;
    void* unused_88;
    void* unused_89;
    void* unused_90;
    void* unused_91;
    void* unused_92;
    void* unused_93;
    void* unused_94;
    void* unused_95;
    void* unused_96;
    void* unused_97;
    void* unused_98;
    void* unused_99;
    void* unused_100;
    void* unused_101;
    void* unused_102;
    void* unused_103;
    void* unused_104;
    void* unused_105;
    void* unused_106;
    void* unused_107;
    void* unused_108;
    void* unused_109;
    void* unused_110;
    void* unused_111;
    void* unused_112;
    void* unused_113;
    void* unused_114;
    void* unused_115;
    void* unused_116;
    void* unused_117;
    void* unused_118;
    void* unused_119;
    void* unused_120;
    void* unused_121;
    void* unused_122;
    void* unused_123;
    void* unused_124;
    void* unused_125;
    void* unused_126;
    void* unused_127;
    void* unused_128;
    void* unused_129;
    void* unused_130;
    void* unused_131;
    void* unused_132;
    void* unused_133;
    void* unused_134;
    void* unused_135;
    void* unused_136;
    void* unused_137;
    void* unused_138;
    void* unused_139;
    void* unused_140;
    void* unused_141;
    void* unused_142;
    void* unused_143;
    void* unused_144;
    void* unused_145;
    void* unused_146;
    void* unused_147;
    void* unused_148;
    void* unused_149;
    void* unused_150;
    void* unused_151;
    void* unused_152;
    void* unused_153;
    void* unused_154;
    void* unused_155;
    void* unused_156;
    void* unused_157;
    void* unused_158;
    void* unused_159;
    void* unused_160;
    void* unused_161;
    void* unused_162;
    void* unused_163;
    void* unused_164;
    void* unused_165;
    void* unused_166;
    jstring (JNICALL *NewStringUTF)(JNIEnv*, const char*);  /* 167 */
    void* unused_168;
    const char* (JNICALL *GetStringUTFChars)(JNIEnv*, jstring, jboolean*);  /* 169 */
    void (JNICALL *ReleaseStringUTFChars)(JNIEnv*, jstring, const char*);  /* 170 */
    jsize (JNICALL *GetArrayLength)(JNIEnv*, jarray);  /* 171 */
    void* unused_172;
    void* unused_173;
    void* unused_174;
    void* unused_175;
    void* unused_176;
    void* unused_177;
    void* unused_178;
    void* unused_179;
    void* unused_180;
    void* unused_181;
    void* unused_182;
    void* unused_183;
    void* unused_184;
    void* unused_185;
    void* unused_186;
    jint* (JNICALL *GetIntArrayElements)(JNIEnv*, jintArray, jboolean*);  /* 187 */
    void* unused_188;
    jfloat* (JNICALL *GetFloatArrayElements)(JNIEnv*, jfloatArray, jboolean*);  /* 189 */
    void* unused_190;
    void* unused_191;
    void* unused_192;
    void* unused_193;
    void* unused_194;
    void (JNICALL *ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint);  /* 195 */
    void* unused_196;
    void (JNICALL *ReleaseFloatArrayElements)(JNIEnv*, jfloatArray, jfloat*, jint);  /* 197 */
    void* unused_198;
    void* unused_199;
    void* unused_200;
    void* unused_201;
    void* unused_202;
    void* unused_203;
    void* unused_204;
    void* unused_205;
    void* unused_206;
    void* unused_207;
    void* unused_208;
    void* unused_209;
    void* unused_210;
    void* unused_211;
    void* unused_212;
    void* unused_213;
    void* unused_214;
    void* unused_215;
    void* unused_216;
    void* unused_217;
    void* unused_218;
    void* unused_219;
    void* unused_220;
    void* unused_221;
    void* unused_222;
    void* unused_223;
    void* unused_224;
    void* unused_225;
    void* unused_226;
    void* unused_227;
    jboolean (JNICALL *ExceptionCheck)(JNIEnv*);  /* 228 */
    jobject (JNICALL *NewDirectByteBuffer)(JNIEnv*, void*, jlong);  /* 229 */
    void* (JNICALL *GetDirectBufferAddress)(JNIEnv*, jobject);  /* 230 */
    jlong (JNICALL *GetDirectBufferCapacity)(JNIEnv*, jobject);  /* 231 */
    void* unused_232;
};

#endif
