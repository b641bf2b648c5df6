#include <hip/hip_runtime.h>
#include <cstdio>
int main(){int a=0,b=0; hipError_t e=hipDeviceGetStreamPriorityRange(&a,&b); printf("rc %d least %d greatest %d\n", (int)e, a, b); return 0;}
