#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define MAXD 32506u
static uint8_t buf[65536+300];
static uint32_t cnt[32768],off[32768],ord[32768],cls[32768];
static int cmpsz(const void*a,const void*b){uint32_t x=*(uint32_t*)a,y=*(uint32_t*)b; if(cnt[x]!=cnt[y])return cnt[x]>cnt[y]?-1:1; return x<y?-1:1;}
static int cmpcls(const void*a,const void*b){uint32_t x=*(uint32_t*)a,y=*(uint32_t*)b; if(cls[x]!=cls[y])return cls[x]>cls[y]?-1:1; return x<y?-1:1;}
int main(int argc,char**argv){
  int mode=atoi(argv[2]); int chain=argc>3?atoi(argv[3]):128;
  FILE*f=fopen(argv[1],"rb"); uint32_t S=65536;
  double s=0,w=0,pos=0,chunks=0;
  static uint16_t mem[65536]; static uint32_t hh[65536], L[65536];
  while(fread(buf,1,S,f)==S){
    uint32_t n=S,m=n-2; memset(cnt,0,sizeof cnt);
    for(uint32_t p=0;p<m;p++){hh[p]=((buf[p]<<10)^(buf[p+1]<<5)^buf[p+2])&0x7fff;cnt[hh[p]]++;}
    for(int h=0;h<32768;h++){ord[h]=h; uint32_t c=cnt[h],l=0; while(c>1){c=(c+1)>>1;l++;} cls[h]= cnt[h]>=128? 99 : l;}
    if(mode==1) qsort(ord,32768,4,cmpsz);
    if(mode==2) qsort(ord,32768,4,cmpcls);
    uint32_t r=0; for(int i=0;i<32768;i++){off[ord[i]]=r;r+=cnt[ord[i]];}
    static uint32_t st[32768]; memcpy(st,off,sizeof st);
    for(uint32_t p=0;p<m;p++) mem[st[hh[p]]++]=p;
    for(uint32_t k=0;k<m;k++){
      uint32_t p=mem[k],h=hh[p],lim=p>MAXD?p-MAXD:0,l=0;
      for(int t=1;t<=chain;t++){int j=(int)k-t; if(j<(int)off[h])break; uint32_t q=mem[j]; if(t==1?(q<(lim>1?lim:1)):(q<=lim))break; l=t;}
      L[k]=l; s+=l; pos++;
    }
    for(uint32_t c=0;c<m;c+=64){uint32_t mx=0; for(uint32_t k=c;k<c+64&&k<m;k++) if(L[k]>mx)mx=L[k]; w+=64.0*mx; chunks++;}
  }
  printf("mode %d chain %d: exact %.1f/pos lockstep %.1f/pos chunks %.0f\n",mode,chain,s/pos,w/pos,chunks);
}
