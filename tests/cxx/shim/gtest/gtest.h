// Minimal GoogleTest-compatible shim (test infrastructure, not product code).
//
// The reference's tests (tests/*.cpp of oksuman/sorting-fhe) are compiled
// UNCHANGED against this engine's headers by tests/cxx/reference_harness.py;
// googletest itself is not in this image (its submodule in the reference is
// empty), so this header provides the subset those files use: TEST, TEST_F,
// typed suites (TYPED_TEST_SUITE / TYPED_TEST), typed-parameterised suites
// (TYPED_TEST_SUITE_P / TYPED_TEST_P /
// REGISTER_TYPED_TEST_SUITE_P / INSTANTIATE_TYPED_TEST_SUITE_P over
// ::testing::Types), FAIL, EXPECT_/ASSERT_ {EQ,NE,LT,LE,GT,GE,NEAR,TRUE,FALSE} with
// streamed messages, AssertionResult, InitGoogleTest, RUN_ALL_TESTS and
// --gtest_filter (':'-separated globs, '-' for negatives).
#pragma once
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <type_traits>
#include <vector>

namespace testing {

class Message {
  public:
    template <class T>
    Message& operator<<(const T& v) {
        ss_ << v;
        return *this;
    }
    std::string str() const { return ss_.str(); }

  private:
    std::ostringstream ss_;
};

class AssertionResult {
  public:
    explicit AssertionResult(bool ok) : ok_(ok) {}
    explicit operator bool() const { return ok_; }
    template <class T>
    AssertionResult& operator<<(const T& v) {
        std::ostringstream s;
        s << v;
        msg_ += s.str();
        return *this;
    }
    const std::string& message() const { return msg_; }

  private:
    bool ok_;
    std::string msg_;
};
inline AssertionResult AssertionSuccess() { return AssertionResult(true); }
inline AssertionResult AssertionFailure() { return AssertionResult(false); }

class Test {
  public:
    virtual ~Test() = default;
    virtual void SetUp() {}
    virtual void TearDown() {}
    virtual void TestBody() = 0;
};

template <class... Ts>
struct Types {};

namespace internal {

struct TestInfo {
    std::string name;  // Suite.Name
    std::function<Test*()> make;
};
inline std::vector<TestInfo>& registry() {
    static std::vector<TestInfo> r;
    return r;
}
inline int& failures() {
    static int f = 0;
    return f;
}
inline std::string& filter() {
    static std::string f = "*";
    return f;
}
inline bool registerTest(const std::string& name, std::function<Test*()> make) {
    registry().push_back({name, std::move(make)});
    return true;
}

inline bool globMatch(const char* p, const char* s) {
    if (!*p) return !*s;
    if (*p == '*') return globMatch(p + 1, s) || (*s && globMatch(p, s + 1));
    if (*p == '?') return *s && globMatch(p + 1, s + 1);
    return *p == *s && globMatch(p + 1, s + 1);
}
inline bool anyMatch(const std::string& pats, const std::string& name) {
    size_t b = 0;
    while (b <= pats.size()) {
        size_t e = pats.find(':', b);
        if (e == std::string::npos) e = pats.size();
        if (e > b && globMatch(pats.substr(b, e - b).c_str(), name.c_str())) return true;
        b = e + 1;
    }
    return false;
}
inline bool& alsoRunDisabled() {
    static bool b = false;
    return b;
}
inline bool selected(const std::string& name) {
    // DISABLED_ suites / tests run only on request, as in googletest
    if (!alsoRunDisabled() && (name.rfind("DISABLED_", 0) == 0 || name.find(".DISABLED_") != std::string::npos ||
                               name.find("/DISABLED_") != std::string::npos))
        return false;
    const std::string& f = filter();
    const size_t dash = f.find('-');
    const std::string pos = dash == std::string::npos ? f : f.substr(0, dash);
    const std::string neg = dash == std::string::npos ? "" : f.substr(dash + 1);
    return anyMatch(pos.empty() ? "*" : pos, name) && !anyMatch(neg, name);
}

template <class T, class = void>
struct Printable : std::false_type {};
template <class T>
struct Printable<T, decltype(void(std::declval<std::ostream&>() << std::declval<const T&>()))> : std::true_type {};
template <class T>
std::string show(const T& v) {
    if constexpr (Printable<T>::value) {
        std::ostringstream s;
        s << v;
        return s.str();
    } else {
        return "<value>";
    }
}

inline std::vector<std::string>& traces();
struct Helper {
    const char* file;
    int line;
    std::string text;
    bool fatal;
    void operator=(const Message& m) const {
        ++failures();
        std::cout << file << ":" << line << ": Failure\n" << text;
        for (const auto& t : traces()) std::cout << "\n  (trace) " << t;
        const std::string extra = m.str();
        if (!extra.empty()) std::cout << "\n" << extra;
        std::cout << std::endl;
    }
};

template <class A, class B>
std::string cmpText(const char* ea, const char* op, const char* eb, const A& a, const B& b) {
    return std::string("Expected: (") + ea + ") " + op + " (" + eb + "), actual: " + show(a) + " vs " + show(b);
}
inline bool toBool(bool b) { return b; }
inline bool toBool(const AssertionResult& r) { return static_cast<bool>(r); }
inline std::string why(const AssertionResult& r) { return r.message(); }
inline std::string why(bool) { return ""; }

}  // namespace internal

inline void InitGoogleTest(int* argc, char** argv) {
    for (int i = 1; argc && i < *argc; ++i)
        if (std::strncmp(argv[i], "--gtest_filter=", 15) == 0)
            internal::filter() = argv[i] + 15;
        else if (std::strcmp(argv[i], "--gtest_also_run_disabled_tests") == 0)
            internal::alsoRunDisabled() = true;
}
inline void InitGoogleTest() {}

}  // namespace testing

inline int RUN_ALL_TESTS() {
    using namespace testing::internal;
    int ran = 0, failedTests = 0;
    for (auto& t : registry()) {
        if (!selected(t.name)) continue;
        ++ran;
        std::cout << "[ RUN      ] " << t.name << std::endl;
        const int before = failures();
        try {
            std::unique_ptr<testing::Test> obj(t.make());
            obj->SetUp();
            if (failures() == before) obj->TestBody();
            obj->TearDown();
        } catch (const std::exception& e) {
            ++failures();
            std::cout << "unexpected exception: " << e.what() << std::endl;
        }
        const bool ok = failures() == before;
        failedTests += !ok;
        std::cout << (ok ? "[       OK ] " : "[  FAILED  ] ") << t.name << std::endl;
    }
    std::cout << "[==========] " << ran << " tests ran, " << failedTests << " failed." << std::endl;
    return failedTests ? 1 : 0;
}

#define SHIM_CAT_(a, b) a##b
#define SHIM_CAT(a, b) SHIM_CAT_(a, b)

#define SHIM_TEST_(suite, name, base)                                                           \
    class SHIM_CAT(suite, SHIM_CAT(_, SHIM_CAT(name, _Test))) : public base {                    \
      public:                                                                                     \
        void TestBody() override;                                                                 \
    };                                                                                            \
    static const bool SHIM_CAT(suite, SHIM_CAT(_, SHIM_CAT(name, _reg))) =                        \
        ::testing::internal::registerTest(#suite "." #name, [] {                                  \
            return static_cast<::testing::Test*>(new SHIM_CAT(suite, SHIM_CAT(_, SHIM_CAT(name, _Test)))()); \
        });                                                                                       \
    void SHIM_CAT(suite, SHIM_CAT(_, SHIM_CAT(name, _Test)))::TestBody()

#define TEST(suite, name) SHIM_TEST_(suite, name, ::testing::Test)
#define TEST_F(fixture, name) SHIM_TEST_(fixture, name, fixture)

// typed-parameterised suites: each TYPED_TEST_P(F, Name) is a class template
// plus a registrar; REGISTER_ collects the names, INSTANTIATE_ walks the types
#define TYPED_TEST_SUITE_P(F) template <class T> struct SHIM_CAT(F, _ShimRegs)
#define TYPED_TEST_P(F, Name)                                                                     \
    template <class gtest_TypeParam_>                                                             \
    class SHIM_CAT(F, SHIM_CAT(_, Name)) : public F<gtest_TypeParam_> {                          \
      public:                                                                                     \
        typedef F<gtest_TypeParam_> TestFixture;                                                  \
        typedef gtest_TypeParam_ TypeParam;                                                       \
        void TestBody() override;                                                                 \
    };                                                                                            \
    struct SHIM_CAT(F, SHIM_CAT(_, SHIM_CAT(Name, _Reg))) {                                       \
        template <class T>                                                                        \
        static void reg(const std::string& prefix) {                                              \
            ::testing::internal::registerTest(prefix + "." #Name, [] {                            \
                return static_cast<::testing::Test*>(new SHIM_CAT(F, SHIM_CAT(_, Name))<T>());    \
            });                                                                                   \
        }                                                                                         \
    };                                                                                            \
    template <class gtest_TypeParam_>                                                             \
    void SHIM_CAT(F, SHIM_CAT(_, Name))<gtest_TypeParam_>::TestBody()

#define SHIM_REG1(F, T, p, a) SHIM_CAT(F, SHIM_CAT(_, SHIM_CAT(a, _Reg)))::template reg<T>(p);
#define SHIM_REG_N(_1, _2, _3, _4, _5, _6, _7, _8, N, ...) N
#define SHIM_REG_1(F, T, p, a) SHIM_REG1(F, T, p, a)
#define SHIM_REG_2(F, T, p, a, ...) SHIM_REG1(F, T, p, a) SHIM_REG_1(F, T, p, __VA_ARGS__)
#define SHIM_REG_3(F, T, p, a, ...) SHIM_REG1(F, T, p, a) SHIM_REG_2(F, T, p, __VA_ARGS__)
#define SHIM_REG_4(F, T, p, a, ...) SHIM_REG1(F, T, p, a) SHIM_REG_3(F, T, p, __VA_ARGS__)
#define SHIM_REG_5(F, T, p, a, ...) SHIM_REG1(F, T, p, a) SHIM_REG_4(F, T, p, __VA_ARGS__)
#define SHIM_REG_6(F, T, p, a, ...) SHIM_REG1(F, T, p, a) SHIM_REG_5(F, T, p, __VA_ARGS__)
#define SHIM_REG_7(F, T, p, a, ...) SHIM_REG1(F, T, p, a) SHIM_REG_6(F, T, p, __VA_ARGS__)
#define SHIM_REG_8(F, T, p, a, ...) SHIM_REG1(F, T, p, a) SHIM_REG_7(F, T, p, __VA_ARGS__)
#define REGISTER_TYPED_TEST_SUITE_P(F, ...)                                                       \
    template <class T>                                                                            \
    struct SHIM_CAT(F, _ShimRegs) {                                                               \
        static void reg(const std::string& p) {                                                   \
            SHIM_REG_N(__VA_ARGS__, SHIM_REG_8, SHIM_REG_7, SHIM_REG_6, SHIM_REG_5, SHIM_REG_4,   \
                       SHIM_REG_3, SHIM_REG_2, SHIM_REG_1)(F, T, p, __VA_ARGS__)                  \
        }                                                                                         \
    }

namespace testing {
namespace internal {
template <template <class> class R, class L>
struct ForTypes;
template <template <class> class R, class... Ts>
struct ForTypes<R, ::testing::Types<Ts...>> {
    static bool run(const std::string& prefix) {
        int i = 0;
        (R<Ts>::reg(prefix + "/" + std::to_string(i++)), ...);
        return true;
    }
};
}  // namespace internal
}  // namespace testing

#define INSTANTIATE_TYPED_TEST_SUITE_P(Prefix, F, TypesList)                                     \
    static const bool SHIM_CAT(SHIM_CAT(Prefix, F), _inst) =                                      \
        ::testing::internal::ForTypes<SHIM_CAT(F, _ShimRegs), TypesList>::run(#Prefix "/" #F)

// typed suites: TYPED_TEST_SUITE(F, Types) names the type list, each
// TYPED_TEST(F, Name) registers itself for every type in it (F/0.Name, ...)
#define TYPED_TEST_SUITE(F, TypesList) typedef TypesList SHIM_CAT(F, _ShimTypes)
#define TYPED_TEST(F, Name)                                                                       \
    template <class gtest_TypeParam_>                                                             \
    class SHIM_CAT(F, SHIM_CAT(_, Name)) : public F<gtest_TypeParam_> {                          \
      public:                                                                                     \
        typedef F<gtest_TypeParam_> TestFixture;                                                  \
        typedef gtest_TypeParam_ TypeParam;                                                       \
        void TestBody() override;                                                                 \
    };                                                                                            \
    template <class T>                                                                            \
    struct SHIM_CAT(F, SHIM_CAT(_, SHIM_CAT(Name, _TReg))) {                                      \
        static void reg(const std::string& prefix) {                                              \
            ::testing::internal::registerTest(prefix + "." #Name, [] {                            \
                return static_cast<::testing::Test*>(new SHIM_CAT(F, SHIM_CAT(_, Name))<T>());    \
            });                                                                                   \
        }                                                                                         \
    };                                                                                            \
    static const bool SHIM_CAT(F, SHIM_CAT(_, SHIM_CAT(Name, _inst))) =                           \
        ::testing::internal::ForTypes<SHIM_CAT(F, SHIM_CAT(_, SHIM_CAT(Name, _TReg))),            \
                                      SHIM_CAT(F, _ShimTypes)>::run(#F);                          \
    template <class gtest_TypeParam_>                                                             \
    void SHIM_CAT(F, SHIM_CAT(_, Name))<gtest_TypeParam_>::TestBody()

// assertions
#define SHIM_ASSERT_(ok, text, fatal) \
    if (ok)                           \
        ;                             \
    else                              \
        SHIM_FAIL_##fatal(text)
#define SHIM_FAIL_1(text) return ::testing::internal::Helper{__FILE__, __LINE__, text, true} = ::testing::Message()
#define SHIM_FAIL_0(text) ::testing::internal::Helper{__FILE__, __LINE__, text, false} = ::testing::Message()
#define SHIM_CMP_(a, op, b, fatal) \
    SHIM_ASSERT_(((a)op(b)), ::testing::internal::cmpText(#a, #op, #b, (a), (b)), fatal)
#define FAIL() SHIM_FAIL_1("Failed")
#define ADD_FAILURE() SHIM_FAIL_0("Failed")
#define EXPECT_EQ(a, b) SHIM_CMP_(a, ==, b, 0)
#define EXPECT_NE(a, b) SHIM_CMP_(a, !=, b, 0)
#define EXPECT_LT(a, b) SHIM_CMP_(a, <, b, 0)
#define EXPECT_LE(a, b) SHIM_CMP_(a, <=, b, 0)
#define EXPECT_GT(a, b) SHIM_CMP_(a, >, b, 0)
#define EXPECT_GE(a, b) SHIM_CMP_(a, >=, b, 0)
#define ASSERT_EQ(a, b) SHIM_CMP_(a, ==, b, 1)
#define ASSERT_NE(a, b) SHIM_CMP_(a, !=, b, 1)
#define ASSERT_LT(a, b) SHIM_CMP_(a, <, b, 1)
#define ASSERT_LE(a, b) SHIM_CMP_(a, <=, b, 1)
#define ASSERT_GT(a, b) SHIM_CMP_(a, >, b, 1)
#define ASSERT_GE(a, b) SHIM_CMP_(a, >=, b, 1)
#define SHIM_NEAR_(a, b, t, fatal)                                                                 \
    SHIM_ASSERT_(std::fabs((double)(a) - (double)(b)) <= (double)(t),                             \
                 ::testing::internal::cmpText(#a, "~=", #b, (a), (b)) + " (tolerance " #t ")", fatal)
#define EXPECT_NEAR(a, b, t) SHIM_NEAR_(a, b, t, 0)
#define ASSERT_NEAR(a, b, t) SHIM_NEAR_(a, b, t, 1)
#define EXPECT_TRUE(c) \
    SHIM_ASSERT_(::testing::internal::toBool(c), std::string("Expected true: " #c " ") + ::testing::internal::why(c), 0)
#define ASSERT_TRUE(c) \
    SHIM_ASSERT_(::testing::internal::toBool(c), std::string("Expected true: " #c " ") + ::testing::internal::why(c), 1)
// SCOPED_TRACE(msg): the message is printed with any failure in its scope
namespace testing {
namespace internal {
inline std::vector<std::string>& traces() {
    static std::vector<std::string> t;
    return t;
}
struct ScopedTrace {
    template <class T>
    explicit ScopedTrace(const T& m) {
        std::ostringstream s;
        s << m;
        traces().push_back(s.str());
    }
    ~ScopedTrace() { traces().pop_back(); }
};
}  // namespace internal
}  // namespace testing
#define SCOPED_TRACE(m) ::testing::internal::ScopedTrace SHIM_CAT(shim_trace_, __LINE__)(m)
#define EXPECT_FALSE(c) SHIM_ASSERT_(!::testing::internal::toBool(c), "Expected false: " #c, 0)
#define ASSERT_FALSE(c) SHIM_ASSERT_(!::testing::internal::toBool(c), "Expected false: " #c, 1)
