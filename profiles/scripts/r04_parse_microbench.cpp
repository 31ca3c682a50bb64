#include <sys/mman.h>
#include <sys/stat.h>
#include <fcntl.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <thread>
#include <vector>
#include <algorithm>
static double now(){return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();}
inline bool fast_line(const char*& p, const char* end, int64_t* va, int64_t* vb) {
  const char* q = p;
  if (q >= end || *q < '0' || *q > '9') return false;
  int64_t x = 0; int nd = 0;
  while (q < end && *q >= '0' && *q <= '9' && nd < 18) x = x * 10 + (*q++ - '0'), ++nd;
  if (q >= end || (*q != ' ' && *q != '\t')) return false;
  while (q < end && (*q == ' ' || *q == '\t')) ++q;
  if (q >= end || *q < '0' || *q > '9') return false;
  int64_t y = 0; nd = 0;
  while (q < end && *q >= '0' && *q <= '9' && nd < 18) y = y * 10 + (*q++ - '0'), ++nd;
  while (q < end && (*q == ' ' || *q == '\t' || *q == '\r')) ++q;
  if (q < end && *q != '\n') return false;
  *va = x; *vb = y; p = q + 1; return true;
}
// unchecked: caller guarantees a '\n' at or before end-1
inline bool fast_line_u(const char*& p, int64_t* va, int64_t* vb) {
  const char* q = p;
  unsigned d = (unsigned char)*q - '0';
  if (d > 9) return false;
  int64_t x = 0; const char* s = q;
  do { x = x * 10 + d; d = (unsigned char)*++q - '0'; } while (d <= 9);
  if (q - s > 18 || (*q != ' ' && *q != '\t')) return false;
  do ++q; while (*q == ' ' || *q == '\t');
  d = (unsigned char)*q - '0';
  if (d > 9) return false;
  int64_t y = 0; s = q;
  do { y = y * 10 + d; d = (unsigned char)*++q - '0'; } while (d <= 9);
  if (q - s > 18) return false;
  while (*q == ' ' || *q == '\t' || *q == '\r') ++q;
  if (*q != '\n') return false;
  *va = x; *vb = y; p = q + 1; return true;
}
int main(int argc,char**argv){
  int fd=open(argv[1],O_RDONLY); struct stat st; fstat(fd,&st); size_t size=st.st_size;
  int nt=atoi(argv[2]); int mode=atoi(argv[3]);
  for(int rep=0;rep<6;rep++){
  double t0=now();
  const char* data=(const char*)mmap(nullptr,size,PROT_READ,MAP_PRIVATE|MAP_POPULATE,fd,0);
  std::vector<size_t> cut(nt+1,size); cut[0]=0;
  for(int t=1;t<nt;t++){size_t c=size*t/nt; while(c<size&&data[c-1]!='\n')++c; cut[t]=c;}
  std::vector<std::vector<int64_t>> A(nt),B(nt); std::vector<std::vector<int32_t>> C(nt);
  std::vector<std::thread> th;
  for(int t=0;t<nt;t++) th.emplace_back([&,t]{
    const char*p=data+cut[t],*end=data+cut[t+1];
    auto&a=A[t];auto&b=B[t]; if(mode<2&&mode!=3){a.reserve((end-p)/12+16); b.reserve((end-p)/12+16);}
    int64_t va,vb,sa=0; const bool sto = mode<2;
    if(mode==3){ auto&c=C[t]; c.resize((end-p)/6+16); size_t k=0; const char* ue = end; while (ue > p && ue[-1] != '\n') --ue;
      while(p<ue){ if(fast_line_u(p,&va,&vb)){c[k]=(int32_t)va;c[k+1]=(int32_t)vb;k+=2;continue;} while(p<end&&*p!='\n')++p; ++p;} c.resize(k); a.push_back(k/2); }
    else if(mode==0){ while(p<end){ if(fast_line(p,end,&va,&vb)){if(sto){a.push_back(va);b.push_back(vb);}else sa+=va^vb;continue;} while(p<end&&*p!='\n')++p; ++p;} }
    else { const char* ue = end; while (ue > p && ue[-1] != '\n') --ue;  // unchecked region
      while(p<ue){ if(fast_line_u(p,&va,&vb)){if(sto){a.push_back(va);b.push_back(vb);}else sa+=va^vb;continue;} while(p<end&&*p!='\n')++p; ++p;}
      while(p<end){ if(fast_line(p,end,&va,&vb)){if(sto){a.push_back(va);b.push_back(vb);}else sa+=va^vb;continue;} while(p<end&&*p!='\n')++p; ++p;} }
  if(!sto) a.push_back(sa); });
  for(auto&x:th)x.join(); (void)0;
  double t1=now(); size_t m=0; for(auto&x:A)m+=x.size();
  printf("mode %d nt %d parse %.4f m %zu\n",mode,nt,t1-t0,m);
  munmap((void*)data,size);
  }
}
